"""Level-1 FPS alone (HREG_LIB selects the library): the register kernel and the pruned kernel over
the spatial index on 16 KITTI-shape clouds, per dependent iteration, plus a bitwise check.

  python tools/fps_sorted_time.py
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from pcd_reg_hregnet_amd import _lib, engine, synthetic  # noqa: E402


def main():
    _lib.load()
    s, d, _, _ = synthetic.lidar_batch(8, 16384, seed0=21)
    pts = torch.cat([torch.from_numpy(s), torch.from_numpy(d)]).cuda().contiguous()
    nb, n, _ = pts.shape
    m = 1024
    st = _lib.stream_handle()
    ws = torch.empty(engine.spatial_index_bytes(nb, n), dtype=torch.uint8, device="cuda")
    a = torch.empty(nb, m, dtype=torch.int32, device="cuda")
    b = torch.empty(nb, m, dtype=torch.int32, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    res = []
    for rep in range(4):
        _lib.call("hreg_spatial_index", pts, nb, n, ws, st)
        ev[0].record()
        _lib.call("hreg_furthest_point_sampling", nb, n, m, pts, None, a, None, st)
        ev[1].record()
        _lib.call("hreg_fps_indexed", nb, n, m, pts, ws, None, b, None, st)
        ev[2].record()
        torch.cuda.synchronize()
        if rep:
            res.append((ev[0].elapsed_time(ev[1]) * 1e3 / (m - 1), ev[1].elapsed_time(ev[2]) * 1e3 / (m - 1)))
    assert torch.equal(a, b), "pruned FPS differs"
    reg = sorted(r[0] for r in res)[1]
    srt = sorted(r[1] for r in res)[1]
    print(f"{os.environ.get('HREG_LIB', 'tree')}: reg {reg:.4f} us/iter, sorted {srt:.4f} us/iter", flush=True)


if __name__ == "__main__":
    main()
