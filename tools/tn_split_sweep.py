"""Weight-gradient GEMM (hreg_gemm_tn: dW = dY^T X, split-R + in-order reduction) timed per
row-split count S on the training step's level-2 / level-3 / head shapes (HIP events, median
of reps), beside the library's own choice and the shape's roofline (f32 MFMA 157.3 TF/s,
HBM 8 TB/s on the compulsory bytes).

usage: python tools/tn_split_sweep.py [--reps 10]"""
import argparse
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pcd_reg_hregnet_amd import _lib  # noqa: E402

# (R, N, K): dW [N][K] of a conv K -> N over R rows (B = 8 per side)
SHAPES = [
    (131072, 64, 68), (131072, 64, 64), (131072, 128, 64), (131072, 64, 384),
    (32768, 128, 132), (32768, 128, 128), (32768, 256, 128), (32768, 128, 768),
    (16384, 512, 528), (16384, 512, 512), (16384, 256, 260), (32768, 256, 268),
    (65536, 128, 140), (65536, 128, 128),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    lib = _lib.load()
    dev = torch.device("cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for R, N, K in SHAPES:
        A = torch.randn(R, N, device=dev)
        B = torch.randn(R, K, device=dev)
        out = torch.empty(N, K, device=dev)
        S0 = lib.hreg_gemm_tn_ws_bytes(R, N, K) // (4 * N * K)
        cands = sorted({s for s in (4, 8, 16, 32, 64, 128, 256, 512, 1024) if R // s >= 64} | {S0})
        ws = torch.empty(max(cands) * N * K, device=dev)
        ref = None
        res = []
        for S in cands:
            ts = []
            for r in range(a.reps + 2):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                rc = lib.hreg_debug_gemm_tn_s(ctypes.c_void_p(A.data_ptr()), N, ctypes.c_void_p(B.data_ptr()), K,
                                              R, N, K, ctypes.c_float(0.0), ctypes.c_void_p(ws.data_ptr()),
                                              ctypes.c_void_p(out.data_ptr()), st, S)
                e1.record()
                assert rc == 0, rc
                if r >= 2:
                    ts.append((e0, e1))
            torch.cuda.synchronize()
            us = statistics.median(x.elapsed_time(y) * 1e3 for x, y in ts)
            if ref is None:
                ref = out.clone()
            err = float((out - ref).abs().max() / ref.abs().max())
            res.append((S, us, err))
        flop = 2.0 * R * N * K
        ideal = max(flop / 157.3e6, 4.0 * R * (N + K) / 8e6)
        best = min(res, key=lambda t: t[1])
        line = "  ".join(f"S={s}:{us:.1f}" + ("*" if s == S0 else "") for s, us, _ in res)
        print(f"R={R:6d} N={N:3d} K={K:3d} ideal {ideal:6.1f} us | {line} | best S={best[0]} "
              f"{best[1]:.1f} us vs default {dict((s, u) for s, u, _ in res)[S0]:.1f} "
              f"| max rel diff {max(e for _, _, e in res):.1e}", flush=True)


if __name__ == "__main__":
    main()
