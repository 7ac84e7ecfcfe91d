"""Build variants of group_split.hip (HREG_SPLIT_EXP 0/1/2) and time levels 2 and 3 at
config-2 sizes.  usage: python tools/split_experiment.py   (GPU box; builds into /tmp)"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from tools.op_bench import timeit  # noqa: E402
from tools.group_bench import LEVELS  # noqa: E402

SRC = os.path.join(REPO, "pcd_reg_hregnet_amd", "csrc", "group_split.hip")


def build(flags, tag):
    out = f"/tmp/splitexp_{tag}.so"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                           "-ffp-contract=off", "-shared", "-fPIC", *flags, SRC, "-o", out])
    return out


def main(variants):
    torch.cuda.init()
    rng = np.random.default_rng(0)
    res = {}
    for tag, flags in variants.items():
        L = ctypes.CDLL(build(flags, tag))
        for name, G, KN, CF, C3, CM2, fl in LEVELS:
            f = getattr(L, f"hreg_group_split_{name}_table_floats")
            f.restype = ctypes.c_int
            nt = f()
            tb = torch.from_numpy(rng.normal(0, 0.05, nt).astype(np.float32)).cuda()
            R = G * KN
            geom = torch.from_numpy(rng.normal(size=(R, 4)).astype(np.float32)).cuda()
            kx = torch.from_numpy(rng.normal(size=(R, 3)).astype(np.float32)).cuda()
            gidx = torch.from_numpy(rng.integers(0, 2 * G, R).astype(np.int32)).cuda()
            feats = torch.from_numpy(np.abs(rng.normal(size=(2 * G, CF))).astype(np.float32)).cuda()
            kp = torch.empty(G, 3, device="cuda")
            att = torch.empty(G, C3, device="cuda")
            desc = torch.empty(G, CM2, device="cuda")
            p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
            st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            fn = getattr(L, f"hreg_group_split_{name}")
            ms = timeit(lambda: fn(p(tb), p(geom), p(kx), p(gidx), p(feats), G, p(kp), p(att),
                                   p(desc), st), reps=20)
            res[f"{tag}_{name}"] = (round(ms, 4), round(fl * G / ms / 1e9, 1))
    print(res)


if __name__ == "__main__":
    main({"base": [], "noldsB": ["-DHREG_SPLIT_EXP=2"], "noA": ["-DHREG_L2_EXP=2"],
          "noA_noB": ["-DHREG_L2_EXP=2", "-DHREG_SPLIT_EXP=2"]})
