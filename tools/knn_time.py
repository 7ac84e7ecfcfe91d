"""Eager timing of the level-1 indexed kNN (hreg_knn_group_indexed, 64 clouds x 16384 points,
1024 centres each, k = 64) and its spatial index; HIP events over 20 launches after 3 warm-up.
    python tools/knn_time.py   (HREG_LIB=... for another build)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pcd_reg_hregnet_amd import _lib, engine, synthetic  # noqa: E402

nb, n, m, k = 64, 16384, 1024, 64
s, d, _, _ = synthetic.lidar_batch(nb // 2, n, seed0=3)
x = torch.from_numpy(np.concatenate([s, d])).cuda()
ws = torch.empty(engine.spatial_index_bytes(nb, n), dtype=torch.uint8, device="cuda")
st = _lib.stream_handle()
_lib.call("hreg_spatial_index", x, nb, n, ws, st)
idx, q = engine.fps_indexed(x, m, ws)
gidx = torch.empty(nb * m * k, dtype=torch.int32, device="cuda")
geom = torch.empty(nb * m * k, 4, device="cuda")
kx = torch.empty(nb * m * k, 3, device="cuda")


def run():
    _lib.call("hreg_knn_group_indexed", q, x, ws, nb, m, n, k, gidx, geom, kx, st)


def index():
    _lib.call("hreg_spatial_index", x, nb, n, ws, st)


for name, fn in (("knn_group_indexed", run), ("spatial_index", index)):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        fn()
    b.record()
    torch.cuda.synchronize()
    print(f"{name}: {a.elapsed_time(b) / 20 * 1e3:.1f} us per launch")
