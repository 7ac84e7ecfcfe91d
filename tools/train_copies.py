"""Where the training step's copy / fill launches come from: one eager Trainer step under
torch.profiler (with Python stacks); every aten copy_ / fill_ / zero_ / clone / cat / contiguous
call grouped by its innermost pcd_reg_hregnet_amd frame, with counts and bytes.

usage: python tools/train_copies.py OUT.txt"""
import collections
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

OPS = ("aten::copy_", "aten::fill_", "aten::zero_", "aten::zeros", "aten::clone", "aten::cat",
       "aten::contiguous", "aten::zeros_like", "aten::new_zeros", "aten::index_select", "aten::add_",
       "aten::mul_", "aten::sum")


def main():
    out = sys.argv[1]
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
    for _ in range(3):
        tr.step(src, dst, gR, gt, next_batch=(src, dst))
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
        tr.step(src, dst, gR, gt, next_batch=(src, dst))
        torch.cuda.synchronize()
    sites = collections.Counter()
    for ev in prof.events():
        if ev.name not in OPS:
            continue
        frame = "?"
        for fr in (ev.stack or []):
            if "pcd_reg_hregnet_amd" in fr or "torch/autograd" in fr or "torch/optim" in fr:
                frame = fr.split("pcd_reg_hregnet_amd/")[-1]
                break
        shapes = ev.input_shapes[0] if ev.input_shapes else None
        sites[(ev.name, frame, str(shapes))] += 1
    lines = [f"{n:5d}  {op:22s} {site}  {shp}" for (op, site, shp), n in sites.most_common()]
    per_op = collections.Counter()
    for (op, _, _), n in sites.items():
        per_op[op] += n
    lines = [f"per op: {dict(per_op)}", ""] + lines
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:60]))


if __name__ == "__main__":
    main()
