"""Level-1 FPS of 16384-point clouds alone: fps_sorted_kernel (hreg_fps_indexed) vs the
small-footprint fps_blocks_kernel<4> (hreg_fps_indexed_lean), per dependent iteration, for a
single batch (16 clouds: the latency path) and the batched stage's 64 / 256 / 768 clouds; bitwise
check.   python tools/fps_lean_time.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pcd_reg_hregnet_amd import _lib, engine, synthetic  # noqa: E402

n, m = 16384, 1024
st = _lib.stream_handle()
for nb in (16, 64, 256, 768):
    s, d, _, _ = synthetic.lidar_batch(8, n, seed0=5)
    one = torch.cat([torch.from_numpy(s), torch.from_numpy(d)]).cuda()
    pts = one.repeat((nb + 15) // 16, 1, 1)[:nb].contiguous()
    ws = torch.empty(engine.spatial_index_bytes(nb, n), dtype=torch.uint8, device="cuda")
    _lib.call("hreg_spatial_index", pts, nb, n, ws, st)
    out = {}
    for name in ("hreg_fps_indexed", "hreg_fps_indexed_lean"):
        idx = torch.empty(nb, m, dtype=torch.int32, device="cuda")
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        times = []
        for rep in range(3):
            ev[0].record()
            _lib.call(name, nb, n, m, pts, ws, None, idx, None, st)
            ev[1].record()
            torch.cuda.synchronize()
            if rep:
                times.append(ev[0].elapsed_time(ev[1]) * 1e3)
        out[name] = (min(times), idx)
    assert torch.equal(out["hreg_fps_indexed"][1], out["hreg_fps_indexed_lean"][1]), "lean FPS differs"
    print(f"{nb} clouds: sorted {out['hreg_fps_indexed'][0]:.0f} us ({out['hreg_fps_indexed'][0] / (m - 1):.3f} us/it), "
          f"lean {out['hreg_fps_indexed_lean'][0]:.0f} us ({out['hreg_fps_indexed_lean'][0] / (m - 1):.3f} us/it)", flush=True)
