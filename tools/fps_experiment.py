"""Build variants of fps.hip (HREG_FPS_EXP / HREG_FPS_S) and time the multi-workgroup
FPS on 65536-point clouds (config 5 level 1).  usage: python tools/fps_experiment.py"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from tools.op_bench import timeit  # noqa: E402

SRC = os.path.join(REPO, "pcd_reg_hregnet_amd", "csrc", "fps.hip")
VARIANTS = {"base": [], "fourlane": ["-DHREG_FPS_EXP=1"], "pad": ["-DHREG_FPS_PAD=16"],
            "sleep": ["-DHREG_FPS_EXP=2"], "S32": ["-DHREG_FPS_S=32"]}


def build(name):
    out = f"/tmp/fpsexp_{name}.so"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                           "-ffp-contract=off", "-shared", "-fPIC", *VARIANTS[name], SRC, "-o", out])
    return out


def main():
    torch.cuda.init()
    rng = np.random.default_rng(0)
    from pcd_reg_hregnet_amd import synthetic
    lid = synthetic.lidar_batch(2, 65536, seed0=60)
    clouds = {"uniform": rng.uniform(-40, 40, (4, 65536, 3)).astype(np.float32),
              "lidar": np.concatenate([lid[0], lid[1]], 0)}
    res = {}
    ref = None
    for name in VARIANTS:
        L = ctypes.CDLL(build(name))
        fn = L.hreg_furthest_point_sampling
        fn.restype = ctypes.c_int
        for cname, c in clouds.items():
            x = torch.from_numpy(c).cuda()
            nb = x.shape[0]
            temp = torch.empty(nb, 65536, device="cuda")
            idx = torch.empty(nb, 1024, dtype=torch.int32, device="cuda")
            st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            call = lambda: fn(nb, 65536, 1024, ctypes.c_void_p(x.data_ptr()),  # noqa: E731
                              ctypes.c_void_p(temp.data_ptr()), ctypes.c_void_p(idx.data_ptr()),
                              None, st)
            res[f"{name}_{cname}_ms"] = round(timeit(call), 4)
            if cname == "lidar":
                got = idx.cpu().numpy()
                ref = got if ref is None else ref
                assert (got == ref).all(), name
    print(res)


if __name__ == "__main__":
    main()
