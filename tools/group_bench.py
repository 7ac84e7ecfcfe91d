"""Time the level-2 / level-3 group kernels: accumulator-chained (group_fused.hip) vs
channel-split (group_split.hip), config-2 sizes (16 clouds).  usage: python tools/group_bench.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pcd_reg_hregnet_amd import _lib  # noqa: E402
from tools.op_bench import timeit  # noqa: E402

# (name, G, KN, CF, C3, CM2, flops per group)
LEVELS = [("l2", 16 * 512, 32, 64, 128, 128,
           2.0 * 32 * (2 * (68 * 64 + 64 * 64 + 64 * 128) + 384 * 64 + 64 * 128)),
          ("l3", 16 * 256, 16, 128, 256, 256,
           2.0 * 16 * (2 * (132 * 128 + 128 * 128 + 128 * 256) + 768 * 128 + 128 * 256))]


def main():
    L = _lib.load()
    rng = np.random.default_rng(0)
    res = {}
    for name, G, KN, CF, C3, CM2, fl in LEVELS:
        nt = getattr(L, f"hreg_group_{name}_table_floats")()
        tb = torch.from_numpy(rng.normal(0, 0.05, nt).astype(np.float32)).cuda()
        R = G * KN
        geom = torch.from_numpy(rng.normal(size=(R, 4)).astype(np.float32)).cuda()
        kx = torch.from_numpy(rng.normal(size=(R, 3)).astype(np.float32)).cuda()
        nrows = G * 2
        gidx = torch.from_numpy(rng.integers(0, nrows, R).astype(np.int32)).cuda()
        feats = torch.from_numpy(np.abs(rng.normal(size=(nrows, CF))).astype(np.float32)).cuda()
        outs = {}
        for impl in ("", "split_"):
            kp = torch.empty(G, 3, device="cuda")
            att = torch.empty(G, C3, device="cuda")
            desc = torch.empty(G, CM2, device="cuda")
            fn = f"hreg_group_{impl}{name}"
            ms = timeit(lambda: _lib.call(fn, tb, geom, kx, gidx, feats, G, kp, att, desc,
                                          _lib.stream_handle()), reps=20)
            res[f"{fn}_ms"] = round(ms, 4)
            res[f"{fn}_tflops"] = round(fl * G / ms / 1e9, 1)
            outs[impl] = (kp, att, desc)
        print(name, "max |diff| (different table grouping -> only timing is meaningful):",
              [float((a - b).abs().max()) for a, b in zip(outs[""], outs["split_"])])
    print(res)


if __name__ == "__main__":
    main()
