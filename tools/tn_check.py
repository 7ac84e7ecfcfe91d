"""gemm_tn outputs on fixed shapes (seeded), saved (first arg 'save PATH') or compared bitwise with a
saved run (first arg 'cmp PATH'), plus HIP-event timings; for A/B of two builds via HREG_LIB."""
import os, sys, statistics
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pcd_reg_hregnet_amd import _lib, train  # noqa: E402

SHAPES = [(524288, 64, 32), (524288, 32, 192), (524288, 32, 32), (524288, 32, 4), (131072, 128, 64),
          (131072, 64, 384), (32768, 256, 128), (32768, 128, 132), (16384, 512, 528), (1000, 36, 20),
          (4100, 68, 64)]


def main():
    mode, path = sys.argv[1], sys.argv[2]
    _lib.load()
    print("library", _lib.LIB_PATH)
    res = {}
    g = torch.Generator(device="cpu").manual_seed(0)
    for R, N, K in SHAPES:
        A = torch.randn(R, N, generator=g).cuda()
        B = torch.randn(R, K, generator=g).cuda()
        out = train.gemm_tn(A, B)
        ts = []
        for _ in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); train.gemm_tn(A, B); e1.record(); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        res[f"{R}_{N}_{K}"] = out.cpu().numpy()
        print(f"R={R} N={N} K={K}: {statistics.median(ts):7.1f} us")
    if mode == "save":
        np.savez(path, **res)
    else:
        ref = np.load(path)
        for k, v in res.items():
            same = np.array_equal(ref[k], v)
            print(k, "bitwise" if same else f"DIFF max {np.abs(ref[k] - v).max():.3e}")
            assert same, k


if __name__ == "__main__":
    main()
