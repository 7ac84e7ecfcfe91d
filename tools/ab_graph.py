"""Paired A/B timing of the bench's graph executor in ONE process (run-to-run box noise of
separate bench processes is +-3 % at --steps 20).  Every variant gets two GraphPipelines,
captured while its switches are set (engine module attributes) and created in mirrored order
(A B B A) to cancel the creation-order bias; the timed rounds then alternate over all of them
exactly as bench.py times one (barrier-free: one GPU).

usage: python tools/ab_graph.py [--steps 12] [--merge 4] [--reps 8] VARIANT [VARIANT ...]
  (--steps: executor forwards of --merge reference batches each, one lane per forward: the
  bench's default graph executor, 48 batches = 12 merged forwards on 12 lanes)
  VARIANT = comma-separated key=value (or "base"): engine.FLAG=0, or probe.nofps1=1 / probe.nostage1=1
  (timing probes, results wrong: the level-1 FPS, or the whole level-1 grouping, replaced by a
  copy of a cached result, to price its share of the step)
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

def _nofps1(engine):
    """engine.fps_indexed (the level-1 FPS over the spatial index, 16384-point clouds) with its
    selection served from a cache (one D2D copy per call) -- a timing probe only"""
    real = engine.fps_indexed
    cache = {}

    def fps_indexed(xyz, npoint, ws, out=None, **kw):
        key = tuple(xyz.shape)
        if key not in cache:
            cache[key] = tuple(t.clone() for t in real(xyz, npoint, ws, **kw))
        if out is None:
            return tuple(t.clone() for t in cache[key])
        for o, c in zip(out, cache[key]):
            o.copy_(c)
        return out
    return fps_indexed


def _nostage1(engine):
    """engine.grouping with level 1 (FPS + spatial-index kNN grouping) served from a cache
    (D2D copies into the caller's buffers) -- a timing probe only"""
    real = engine.grouping
    cache = {}

    def grouping(xyz, lvl, weights=None, out=None, ws=None, sample=None, **kw):
        if lvl != 0 or sample is not None or xyz.shape[1] != bench.POINTS:
            return real(xyz, lvl, weights, out, ws, sample, **kw)
        key = tuple(xyz.shape)
        if key not in cache:
            cache[key] = tuple(t.clone() for t in real(xyz, lvl, weights, None, None, None))
        if out is None:
            return tuple(t.clone() for t in cache[key])
        for o, c in zip(out[:5], cache[key]):
            o.copy_(c)
        return tuple(out[:5])
    return grouping


def apply(variant, lib, engine):
    """set a variant's switches; returns the undo list"""
    undo = []
    if variant == "base":
        return undo
    for kv in variant.split(","):
        k, v = kv.split("=")
        if k.startswith("engine."):
            name = k[len("engine."):]
            old = getattr(engine, name)
            setattr(engine, name, type(old)(int(v)) if isinstance(old, (bool, int)) else v)
            undo.append(("engine", name, old))
        elif k == "probe.nostage1" and int(v):
            undo.append(("engine", "grouping", engine.grouping))
            engine.grouping = _nostage1(engine)
        elif k == "alt.torchcopy" and int(v):  # (r6: the front copies through torch._foreach_copy_)
            undo.append(("engine", "copy_many", engine.copy_many))
            engine.copy_many = lambda dsts, srcs: torch._foreach_copy_(list(dsts), list(srcs))
        elif k == "probe.nofps1" and int(v):
            undo.append(("engine", "fps_indexed", engine.fps_indexed))
            engine.fps_indexed = _nofps1(engine)
        else:
            raise ValueError(f"unknown switch {k}")
    return undo


def revert(undo, lib, engine):
    for kind, k, old in reversed(undo):
        setattr(engine, k, old)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--merge", type=int, default=bench.HREGNET_MERGE)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    from pcd_reg_hregnet_amd import _lib, engine
    lib = _lib.load()
    dev = torch.device("cuda")
    net = bench.make_model(dev)
    P = net.prepared(dev)
    s, d, _, _ = bench.shard_batch(0, bench.PAIRS_PER_GPU * a.merge, bench.POINTS)
    sb = bench.PAIRS_PER_GPU if a.merge > 1 else None
    src, dst = torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev)
    # every variant twice, created in mirrored order (A B ... B A): pipelines created earlier
    # measured ~3-4 % faster than later ones in the same process (the same variant in first and
    # second position, tools/ab_graph.py base base), so a single creation order biases the A/B
    order = list(a.variants) + list(a.variants)[::-1]
    pipes = []
    with torch.no_grad():
        for v in order:
            undo = apply(v, lib, engine)
            engine.grouping(torch.cat([src, dst], 0), 0)  # (fills a probe's cache uncaptured)
            g = engine.GraphPipeline(P, src, dst, lanes=a.steps, sub_batch=sb)
            g.prepare(a.warmup)
            g.prepare(a.steps)
            g.run_forwards(a.warmup, stream=True)
            g.run_forwards(a.steps, stream=True)  # one untimed round each
            g.prime()  # (front streaming: the timed rounds replay the streamed graphs, as bench.py's)
            torch.cuda.synchronize()
            revert(undo, lib, engine)
            pipes.append(g)
    times = {v: [] for v in a.variants}
    inst = [[] for _ in order]  # per created instance (the creation-order bias)
    with torch.no_grad():
        for r in range(a.reps):
            idxs = list(range(len(order))) if r % 2 == 0 else list(range(len(order)))[::-1]
            for i in idxs:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                pipes[i].run_forwards(a.steps, stream=True)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / a.steps * 1e3
                times[order[i]].append(ms)
                inst[i].append(ms)
            print(f"rep {r}: " + "  ".join(f"{order[i]}#{i} {inst[i][-1]:.4f}" for i in range(len(order))),
                  flush=True)
    print("per instance (creation order):",
          [(order[i], round(statistics.median(inst[i]), 4)) for i in range(len(order))])
    base = statistics.median(times[a.variants[0]])
    out = {}
    for v in a.variants:
        med = statistics.median(times[v])
        out[v] = {"ms_per_step_median": round(med, 4), "pairs_per_s": round(bench.PAIRS_PER_GPU * a.merge / med * 1e3, 1),
                  "vs_first": round(base / med, 4), "all": [round(t, 4) for t in times[v]]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
