"""Paired A/B timing of the bench's graph executor in ONE process (run-to-run box noise of
separate bench processes is +-3 % at --steps 20).  Every variant gets its own GraphPipeline,
captured while its switches are set (hreg_debug_set keys, engine module attributes); the
timed rounds then alternate A B A B ... exactly as bench.py times one (barrier-free: one GPU).

usage: python tools/ab_graph.py [--steps 20] [--reps 8] VARIANT [VARIANT ...]
  VARIANT = comma-separated key=value (or "base"): fps_track=1,fps_pad_kb=140,engine.FLAG=0
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

DBG = {"fps_track": 1, "fps_pad_kb": 2}


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
        else:
            prev = lib.hreg_debug_set(DBG[k], int(v))
            undo.append(("dbg", DBG[k], prev))
    return undo


def revert(undo, lib, engine):
    for kind, k, old in reversed(undo):
        if kind == "engine":
            setattr(engine, k, old)
        else:
            lib.hreg_debug_set(k, old)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    from pcd_reg_hregnet_amd import _lib, engine
    lib = _lib.load()
    dev = torch.device("cuda")
    net = bench.make_model(dev)
    P = net.prepared(dev)
    s, d, _, _ = bench.shard_batch(0, bench.PAIRS_PER_GPU, bench.POINTS)
    src, dst = torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev)
    pipes = []
    with torch.no_grad():
        for v in a.variants:
            undo = apply(v, lib, engine)
            g = engine.GraphPipeline(P, src, dst, lanes=a.steps)
            g.prepare(a.warmup)
            g.prepare(a.steps)
            g.run_forwards(a.warmup, stream=True)
            g.run_forwards(a.steps, stream=True)  # one untimed round each
            torch.cuda.synchronize()
            revert(undo, lib, engine)
            pipes.append(g)
    times = {v: [] for v in a.variants}
    with torch.no_grad():
        for r in range(a.reps):
            order = a.variants if r % 2 == 0 else a.variants[::-1]
            for v, g in ((v, pipes[a.variants.index(v)]) for v in order):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                g.run_forwards(a.steps, stream=True)
                torch.cuda.synchronize()
                times[v].append((time.perf_counter() - t0) / a.steps * 1e3)
            print(f"rep {r}: " + "  ".join(f"{v} {times[v][-1]:.4f}" for v in a.variants), flush=True)
    base = statistics.median(times[a.variants[0]])
    out = {}
    for v in a.variants:
        med = statistics.median(times[v])
        out[v] = {"ms_per_step_median": round(med, 4), "pairs_per_s": round(bench.PAIRS_PER_GPU / med * 1e3, 1),
                  "vs_first": round(base / med, 4), "all": [round(t, 4) for t in times[v]]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
