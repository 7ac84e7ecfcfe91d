"""Level-1 FPS geometry A/B (n = 16384, m = 1024): 16 waves x 16 slots per lane
vs 8 waves x 32 slots (the default since r2; HREG_FPS_L1_1024 selects 16 x 16, read by
choose_geometry on every launch).
Checks the two index sets are identical, times b = 16 clouds (one step) and b = 768
(the graph executor's batched level-1 stage: 48 lanes x 16 clouds).

usage: python tools/micro/fps_l1_geom.py
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from pcd_reg_hregnet_amd import _lib, engine, synthetic  # noqa: E402
from tools.op_bench import timeit  # noqa: E402


def run(xyz, flag):
    if flag:
        os.environ.pop("HREG_FPS_L1_1024", None)
    else:
        os.environ["HREG_FPS_L1_1024"] = "1"
    out = engine.fps(xyz, 1024)
    torch.cuda.synchronize()
    ms = timeit(lambda: engine.fps(xyz, 1024), reps=7, warm=1)
    return out[0].clone(), ms


def main():
    _lib.load()
    s, d, _, _ = synthetic.lidar_batch(8, 16384, seed0=11)
    one = torch.from_numpy(np.concatenate([s, d])).cuda()
    big = one.repeat(48, 1, 1).contiguous()
    for name, xyz in (("b16", one), ("b768", big)):
        res = []
        for flag in (0, 1, 0, 1):
            idx, ms = run(xyz, flag)
            res.append((flag, idx, ms))
        same = all(torch.equal(res[0][1], r[1]) for r in res)
        print(f"{name}: default {res[0][2]:.3f}/{res[2][2]:.3f} ms, 8x32 {res[1][2]:.3f}/"
              f"{res[3][2]:.3f} ms, idx identical: {same}", flush=True)
        assert same


if __name__ == "__main__":
    main()
