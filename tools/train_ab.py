"""Paired A/B timing of the training step (bench.py --model train's Trainer) in ONE process:
blocks of --steps steps alternate between variants (module attribute switches, e.g.
train.DIRECT_GRAD=0), --reps times each; medians of ms/step.

usage: python tools/train_ab.py [--steps 6] [--reps 6] VARIANT [VARIANT ...]
  VARIANT = "base" or comma-separated module.ATTR=int (module in pcd_reg_hregnet_amd)"""
import argparse
import importlib
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def setter(variant):
    sets = []
    if variant != "base":
        for kv in variant.split(","):
            k, v = kv.split("=")
            mod, attr = k.rsplit(".", 1)
            m = importlib.import_module(f"pcd_reg_hregnet_amd.{mod}")
            old = getattr(m, attr)
            sets.append((m, attr, type(old)(int(v)), old))
    return sets


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
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
    nxt = (src, dst)
    sets = {v: setter(v) for v in a.variants}
    times = {v: [] for v in a.variants}
    for r in range(a.reps + 1):
        order = a.variants if r % 2 == 0 else a.variants[::-1]
        for v in order:
            for m, attr, new, _ in sets[v]:
                setattr(m, attr, new)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                tr.step(src, dst, gR, gt, next_batch=nxt)
            torch.cuda.synchronize()
            if r > 0:  # (rep 0 warms every variant)
                times[v].append((time.perf_counter() - t0) / a.steps * 1e3)
            for m, attr, _, old in sets[v]:
                setattr(m, attr, old)
        if r > 0:
            print(f"rep {r}: " + "  ".join(f"{v} {times[v][-1]:.3f}" for v in a.variants), flush=True)
    base = statistics.median(times[a.variants[0]])
    print(json.dumps({v: {"ms_per_step_median": round(statistics.median(t), 3),
                          "pairs_per_s": round(bench.PAIRS_PER_GPU / statistics.median(t) * 1e3, 1),
                          "vs_first": round(base / statistics.median(t), 4)} for v, t in times.items()}))


if __name__ == "__main__":
    main()
