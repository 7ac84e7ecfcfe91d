"""hreg_ts_gemm timing per shape (HIP events, median of 20): usage python tools/ts_micro.py"""
import os, sys, statistics
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pcd_reg_hregnet_amd import _lib  # noqa: E402

SHAPES = [(524288, 32, 32), (524288, 32, 64), (524288, 64, 32), (524288, 192, 32), (524288, 32, 192),
          (131072, 64, 128), (32768, 256, 256)]


def main():
    _lib.load()
    print("library", _lib.LIB_PATH)
    for R, N, K in SHAPES:
        x = torch.randn(R, K, device="cuda")
        W = torch.randn(N, K, device="cuda")
        out = torch.empty(R, N, device="cuda")
        f = lambda: _lib.call("hreg_ts_gemm", x, K, R, K, W, 0, N, None, None, 0, out, N, _lib.stream_handle())
        for _ in range(3):
            f()
        ts = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); f(); e1.record(); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        us = statistics.median(ts)
        print(f"R={R} N={N} K={K}: {us:7.1f} us  {2*R*N*K/us/1e6:6.1f} TF/s  {4*R*(N+K)/us/1e3:6.0f} GB/s")


if __name__ == "__main__":
    main()
