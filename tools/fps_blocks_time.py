"""Large-cloud level-1 FPS alone (HREG_LIB selects the library): hreg_fps_indexed (fps_blocks_kernel)
against the cluster kernel on NB KITTI-shape clouds of N points, per dependent iteration, plus a
bitwise check.   python tools/fps_blocks_time.py [N] [NB]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from pcd_reg_hregnet_amd import _lib, engine, synthetic  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    _lib.load()
    s, d, _, _ = synthetic.lidar_batch(nb // 2, n, seed0=21)
    pts = torch.cat([torch.from_numpy(s), torch.from_numpy(d)]).cuda().contiguous()
    m = 1024
    st = _lib.stream_handle()
    ws = torch.empty(engine.spatial_index_bytes(nb, n), dtype=torch.uint8, device="cuda")
    temp = torch.empty(nb, n, device="cuda")
    a = torch.empty(nb, m, dtype=torch.int32, device="cuda")
    b = torch.empty(nb, m, dtype=torch.int32, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    res = []
    for rep in range(4):
        ev[0].record()
        _lib.call("hreg_spatial_index", pts, nb, n, ws, st)
        ev[1].record()
        _lib.call("hreg_fps_indexed", nb, n, m, pts, ws, None, b, None, st)
        ev[2].record()
        _lib.call("hreg_fps_bounded", nb, n, m, pts, temp, a, None, 1, st)
        ev[3].record()
        torch.cuda.synchronize()
        if rep:
            res.append([ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(3)])
    assert torch.equal(a, b), "pruned FPS differs"
    med = [sorted(r[i] for r in res)[1] for i in range(3)]
    print(f"{os.path.basename(os.environ.get('HREG_LIB', 'tree'))}: n {n} x {nb}: index {med[0]:.1f} us, "
          f"blocks {med[1] / (m - 1):.4f} us/iter, cluster {med[2] / (m - 1):.4f} us/iter", flush=True)


if __name__ == "__main__":
    main()
