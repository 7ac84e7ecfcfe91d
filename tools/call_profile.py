"""Per-call HIP-event timings of one serial B=8 forward (every C-ABI launch and GEMM).

usage: python tools/call_profile.py [--batch 8] [--points 16384] [--reps 3]
Prints each call with its duration (median over reps) and a per-entry summary.
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pcd_reg_hregnet_amd import _lib, engine, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--points", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda")
    _lib.load()
    net = bench.make_model(dev)
    P = net.prepared(dev)
    s, d, _, _ = synthetic.lidar_batch(args.batch, args.points, seed0=0)
    src, dst = torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()
    with torch.no_grad():
        for _ in range(2):
            engine.hregnet_forward(P, src, dst)
    torch.cuda.synchronize()
    orig_gemm, orig_call = _lib.gemm, engine.call
    rec = []

    def timed(name, fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        rec.append((name, e0, e1))

    def gemm(g):
        timed(f"gemm R={g.R} N={g.N} K={g.K} b={g.batch}", lambda: orig_gemm(g))

    def call(name, *a):
        timed(name, lambda: orig_call(name, *a))
    _lib.gemm, engine.call = gemm, call
    runs = []
    with torch.no_grad():
        for _ in range(args.reps):
            rec.clear()
            engine.hregnet_forward(P, src, dst)
            torch.cuda.synchronize()
            runs.append([(n, a.elapsed_time(b) * 1e3) for n, a, b in rec])
    _lib.gemm, engine.call = orig_gemm, orig_call
    med = [(runs[0][i][0], sorted(r[i][1] for r in runs)[len(runs) // 2])
           for i in range(len(runs[0]))]
    tot = sum(t for _, t in med)
    for n, t in med:
        print(f"{t:9.1f} us  {n}")
    summ = collections.defaultdict(float)
    for n, t in med:
        summ[n.split(" ")[0]] += t
    print(f"--- total {tot / 1e3:.3f} ms over {len(med)} calls")
    for n, t in sorted(summ.items(), key=lambda x: -x[1]):
        print(f"{t:9.1f} us  {100 * t / tot:5.1f} %  {n}")


if __name__ == "__main__":
    main()
