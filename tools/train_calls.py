"""Per-call device time of one eager training step (bench.py --model train's Trainer, one
stream): every library entry the step makes, timed with HIP events around a synchronised call,
grouped by entry name and integer arguments (the shapes), sorted by total time.

usage: python tools/train_calls.py OUT.txt"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    out = sys.argv[1]
    from pcd_reg_hregnet_amd import _lib, engine, train, train_graph, trainer, weights
    from pcd_reg_hregnet_amd.models import HRegNet
    _lib.load()
    dev = torch.device("cuda")
    net = HRegNet(bench._Args())
    net.load_state_dict(weights.make_state_dict(net.state_dict(), seed=0, pretrained_feats=True))
    tr = trainer.Trainer(net.to(dev), lr=1e-3, alpha=1.0)
    trainer.TWO_STREAM = False
    s, d, Rg, tg = bench.shard_batch(0, bench.PAIRS_PER_GPU, bench.POINTS)
    src, dst = torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev)
    gR, gt = torch.from_numpy(Rg).to(dev), torch.from_numpy(tg).to(dev)
    for _ in range(2):
        tr.step(src, dst, gR, gt)
    torch.cuda.synchronize()

    real = _lib.call
    rec = collections.defaultdict(lambda: [0, 0.0])

    def timed(name, *args):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        real(name, *args)
        e1.record()
        e1.synchronize()
        key = (name, tuple(a for a in args if isinstance(a, int) and not isinstance(a, bool))[:8])
        rec[key][0] += 1
        rec[key][1] += e0.elapsed_time(e1)

    mods = [_lib, train, train_graph, engine]
    saved = [(m, getattr(m, "call", None)) for m in mods]
    for m in mods:
        if getattr(m, "call", None) is real:
            m.call = timed
    _lib.call = timed
    try:
        torch.cuda.synchronize()
        tr.step(src, dst, gR, gt)
        torch.cuda.synchronize()
    finally:
        for m, c in saved:
            if c is not None:
                m.call = c
    tot = sum(v[1] for v in rec.values())
    byname = collections.defaultdict(lambda: [0, 0.0])
    for (n, _), (c, t) in rec.items():
        byname[n][0] += c
        byname[n][1] += t
    lines = [f"total timed {tot:.3f} ms over {sum(v[0] for v in rec.values())} calls", "", "by entry:"]
    lines += [f"{t:8.3f} ms {c:5d}  {n}" for n, (c, t) in sorted(byname.items(), key=lambda kv: -kv[1][1])]
    lines += ["", "by entry and integer arguments:"]
    lines += [f"{t:8.3f} ms {c:4d}  {n} {args}" for (n, args), (c, t) in
              sorted(rec.items(), key=lambda kv: -kv[1][1])[:120]]
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:70]))


if __name__ == "__main__":
    main()
