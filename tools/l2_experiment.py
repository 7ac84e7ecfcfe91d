"""Build variants of group_l2.hip (HREG_L2_EXP=0/1/2) and time each on random inputs.

  0: the product kernel; 1: no epilogues / row reductions (MFMA + fragment loads);
  2: also no fragment loads (MFMA issue structure only).
usage: python tools/l2_experiment.py   (on the GPU box; builds into /tmp)
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from tools.op_bench import timeit  # noqa: E402

SRC = os.path.join(REPO, "pcd_reg_hregnet_amd", "csrc", "group_fused.hip")


def build(exp):
    out = f"/tmp/l2exp_{exp}.so"
    flags = {"nt": ["-DHREG_ROWS_NT=1"]}.get(exp, [f"-DHREG_L2_EXP={exp}"])
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                           "-ffp-contract=off", "-shared", "-fPIC", *flags, SRC, "-o", out])
    return out


def main():
    torch.cuda.init()
    rng = np.random.default_rng(0)
    b = 16
    G = b * 512
    res = {}
    for exp in (0, 1, 2, 3):
        L = ctypes.CDLL(build(exp))
        L.hreg_group_l2_table_floats.restype = ctypes.c_int
        nt = L.hreg_group_l2_table_floats()
        tb = torch.from_numpy(rng.normal(0, 0.1, nt).astype(np.float32)).cuda()
        geom = torch.from_numpy(rng.normal(size=(G * 32, 4)).astype(np.float32)).cuda()
        kx = torch.from_numpy(rng.normal(size=(G * 32, 3)).astype(np.float32)).cuda()
        gidx = torch.from_numpy(rng.integers(0, b * 1024, G * 32).astype(np.int32)).cuda()
        feats = torch.from_numpy(rng.normal(size=(G * 32, 64)).astype(np.float32)).cuda()
        kp = torch.empty(G, 3, device="cuda")
        att = torch.empty(G, 128, device="cuda")
        desc = torch.empty(G, 128, device="cuda")
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        fn = lambda: L.hreg_group_l2(p(tb), p(geom), p(kx), p(gidx), p(feats), G, p(kp), p(att),  # noqa: E731
                                     p(desc), st)
        ms = timeit(fn)
        flops = 2.0 * 32 * (2 * (68 * 64 + 64 * 64 + 64 * 128) + 384 * 64 + 64 * 128) * G
        res[exp] = (round(ms, 4), round(flops / ms / 1e9, 1))
    print(res)


if __name__ == "__main__":
    main()
