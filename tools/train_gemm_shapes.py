"""Per-call shapes and HIP-event times of the training step's GEMMs (forward / input-gradient
hreg_gemm, weight-gradient hreg_gemm_tn) and BN passes, one B=8 step after 2 warm-up steps.
usage: python tools/train_gemm_shapes.py"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    from pcd_reg_hregnet_amd import _lib, trainer, weights
    from pcd_reg_hregnet_amd.models import HRegNet
    _lib.load()
    dev = torch.device("cuda")
    net = HRegNet(bench._Args())
    net.load_state_dict(weights.make_state_dict(net.state_dict(), seed=0, pretrained_feats=True))
    tr = trainer.Trainer(net.to(dev), lr=1e-3, alpha=1.0)
    s, d, Rg, tg = bench.shard_batch(0, bench.PAIRS_PER_GPU, bench.POINTS)
    src, dst = torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev)
    gR, gt = torch.from_numpy(Rg).to(dev), torch.from_numpy(tg).to(dev)
    for _ in range(2):
        tr.step(src, dst, gR, gt)
    torch.cuda.synchronize()
    rec = []
    og, oc = _lib.gemm, _lib.call

    def ev():
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def gemm(g):
        e0 = ev()
        og(g)
        rec.append(("gemm", (g.R, g.N, g.K), e0, ev()))

    def call(name, *a):
        e0 = ev()
        oc(name, *a)
        if name in ("hreg_gemm_tn", "hreg_bn_stats", "hreg_bn_apply", "hreg_bn_backward", "hreg_transpose",
                    "hreg_ts_gemm"):
            shape = ((a[4], a[5], a[6]) if name == "hreg_gemm_tn" else (a[2], a[6], a[3]) if name == "hreg_ts_gemm"
                     else (a[1], a[2]) if name != "hreg_bn_backward" else (a[3], a[4]))
            rec.append((name[5:], shape, e0, ev()))
    _lib.gemm, _lib.call = gemm, call
    tr.step(src, dst, gR, gt)
    torch.cuda.synchronize()
    _lib.gemm, _lib.call = og, oc
    agg = collections.defaultdict(lambda: [0, 0.0])
    tot = collections.defaultdict(float)
    for kind, shape, e0, e1 in rec:
        us = e0.elapsed_time(e1) * 1e3
        agg[(kind, shape)][0] += 1
        agg[(kind, shape)][1] += us
        tot[kind] += us
    for (kind, shape), (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        flop = 2.0 * shape[0] * shape[1] * shape[2] if kind in ("gemm", "gemm_tn", "ts_gemm") else 0
        byts = 4.0 * shape[0] * (shape[1] + shape[2]) if kind in ("gemm", "gemm_tn", "ts_gemm") else 0
        print(f"{kind:12s} {str(shape):24s} x{n:3d}  {us / n:8.1f} us/call  {us / 1e3:7.3f} ms"
              + (f"  {flop * n / us / 1e6:6.1f} TF/s  {byts * n / us / 1e3:6.2f} GB/s(min bytes)" if flop else ""))
    print({k: round(v / 1e3, 3) for k, v in tot.items()})


if __name__ == "__main__":
    main()
