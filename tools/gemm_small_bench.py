"""Standalone timing of the forward's short-K GEMM shapes (B = 8) on hreg_gemm, back to
back (HIP events, median of 50): separates the kernel's own time from the in-forward one.
usage: python tools/gemm_small_bench.py   (HREG_GEMM_WAVE=0/1 selects the kernel)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pcd_reg_hregnet_amd import _lib, engine  # noqa: E402
from tools.op_bench import timeit  # noqa: E402

SHAPES = [(16384, 128, 64, 1), (8192, 256, 128, 1), (4096, 256, 256, 1), (2048, 512, 256, 2),
          (4096, 256, 128, 2), (8192, 128, 64, 2)]


def main():
    _lib.load()
    torch.manual_seed(0)
    for R, N, K, b in SHAPES:
        A = torch.randn(b * R, K, device="cuda")
        lin = engine.Lin(torch.randn(N, K, device="cuda") * 0.1, torch.ones(N, device="cuda"),
                         torch.zeros(N, device="cuda"), False)
        out = torch.empty(b * R, N, device="cuda")
        if b == 1:
            f = lambda: engine.gemm([engine._seg(A, 0, K, ld=K)], lin, R, out=out)  # noqa: E731
        else:
            W2 = torch.randn(2, N, K, device="cuda") * 0.1
            lin2 = engine.Lin(W2, lin.alpha, lin.beta, False)
            o2 = out.view(2, R, N)
            f = lambda: engine._gemm_batched_desc(lin2, A, R, K, o2)  # noqa: E731
        us = timeit(f, reps=50, warm=5) * 1e3
        print(f"R={R:6d} N={N:4d} K={K:4d} batch={b}  {us:7.1f} us  {2.0 * R * N * K * b / us / 1e6:6.1f} TF/s",
              flush=True)
    # cosine shape: B=8 pairs of 256 x 256 x 256
    a, bb = torch.randn(8 * 256, 256, device="cuda"), torch.randn(8 * 256, 256, device="cuda")
    na, nb = a.norm(dim=1), bb.norm(dim=1)
    S = torch.empty(8, 256, 256, device="cuda")
    us = timeit(lambda: engine.cosine_gemm(a, bb, na, nb, 8, 256, 256, 256, S), reps=50, warm=5) * 1e3
    print(f"cosine 8 x 256 x 256 x 256  {us:7.1f} us")


if __name__ == "__main__":
    main()
