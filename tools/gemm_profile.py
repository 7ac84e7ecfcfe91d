"""Per-launch GEMM shapes and achieved TFLOP/s for one B=8 forward (HIP events)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pcd_reg_hregnet_amd import _lib, engine, synthetic  # noqa: E402


def main():
    dev = torch.device("cuda")
    _lib.load()
    net = bench.make_model(dev)
    P = net.prepared(dev)
    s, d, _, _ = synthetic.lidar_batch(8, 16384, seed0=0)
    src, dst = torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()
    rec = []
    orig = _lib.gemm

    def gemm(g):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        orig(g)
        e1.record()
        rec.append((g.R, g.N, g.K, g.batch, g.nseg, e0, e1))
    for _ in range(3):
        engine.hregnet_forward(P, src, dst)
    torch.cuda.synchronize()
    _lib.gemm = gemm
    rec.clear()
    engine.hregnet_forward(P, src, dst)
    torch.cuda.synchronize()
    tot = 0.0
    for R, N, K, b, ns, e0, e1 in rec:
        ms = e0.elapsed_time(e1)
        tot += ms
        tf = 2.0 * R * N * K * b / (ms * 1e-3) / 1e12
        print(f"R={R:8d} N={N:4d} K={K:4d} batch={b} segs={ns}  {ms * 1e3:7.1f} us  {tf:6.1f} TF/s")
    print(f"total {tot:.3f} ms over {len(rec)} GEMMs")


if __name__ == "__main__":
    main()
