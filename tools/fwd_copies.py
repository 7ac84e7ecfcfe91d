"""Python call sites of tensor copies in one eager HRegNet forward (the bench's merged
executor forward, 4 x 8 pairs): every builtin copy_ / clone / contiguous / cat / stack / to /
repeat / zeros call made from package code, counted by caller line (sys.setprofile).  The
graph executor replays these as __amd_rocclr_copyBuffer / fill nodes.

usage: python tools/fwd_copies.py OUT.txt"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

NAMES = {"copy_", "clone", "contiguous", "cat", "stack", "to", "repeat", "zeros", "zeros_like",
         "_foreach_copy_", "index_select", "full", "empty_like", "fill_", "zero_"}


def main():
    out = sys.argv[1]
    from pcd_reg_hregnet_amd import _lib, engine
    _lib.load()
    dev = torch.device("cuda")
    net = bench.make_model(dev, "hregnet")
    P = net.prepared(dev)
    B, merge = bench.PAIRS_PER_GPU, bench.HREGNET_MERGE
    s, d, _, _ = bench.shard_batch(0, B * merge, bench.POINTS)
    src, dst = torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev)
    with torch.no_grad():
        for _ in range(2):
            engine.hregnet_forward(P, src, dst, sub_batch=B)
        torch.cuda.synchronize()
        sites = collections.Counter()

        def prof(frame, event, arg):
            if event == "c_call" and getattr(arg, "__name__", "") in NAMES:
                f = frame
                if "pcd_reg_hregnet_amd" in f.f_code.co_filename:
                    sites[(arg.__name__, os.path.basename(f.f_code.co_filename), f.f_lineno,
                           f.f_code.co_name)] += 1
        sys.setprofile(prof)
        try:
            engine.hregnet_forward(P, src, dst, sub_batch=B)
        finally:
            sys.setprofile(None)
        torch.cuda.synchronize()
    lines = [f"{n:4d}  {op:14s} {fn}:{ln} ({co})" for (op, fn, ln, co), n in sites.most_common()]
    lines = [f"{sum(sites.values())} calls"] + lines
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:80]))


if __name__ == "__main__":
    main()
