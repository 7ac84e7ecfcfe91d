"""Training trajectory of our HIP trainer (trainer.Trainer, Adam lr 1e-3) on one fixed batch,
next to the reference's own fp32 / float64 trajectories (tests/golden/train_traj_*.npz, made
by tests/golden/make_golden.py --traj-only [--traj-c4]).

  python tools/train_traj.py [--fixture train_traj_b8_n16384.npz] [--steps 10]
         [--sim torch64]   # the cosine-similarity op replaced by float64 torch autograd

Prints one JSON line: our per-step loss, the reference's, and their spread.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def sim_torch64(a, b, kidx, nb, N1, N2):
    """layers.py:290-313 in float64 torch autograd (cos, row / column max normalisation,
    the gather at the descriptor kNN), cast back to fp32."""
    C = a.shape[1]
    A, Bm = a.double().view(nb, N1, C), b.double().view(nb, N2, C)
    S = torch.bmm(A, Bm.transpose(1, 2)) / (A.norm(dim=-1)[:, :, None] * Bm.norm(dim=-1)[:, None, :]
                                            + 1e-6)
    rn = S / (S.max(2, keepdim=True)[0] + 1e-6)
    cn = S / (S.max(1, keepdim=True)[0] + 1e-6)
    ki = kidx.long().view(nb, N1, -1)
    bi = torch.arange(nb, device=a.device)[:, None, None]
    ii = torch.arange(N1, device=a.device)[:, None][None]
    return torch.stack([rn[bi, ii, ki], cn[bi, ii, ki]], -1).view(-1, 2).float()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fixture", default="train_traj_b2_n2048.npz")
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--sim", choices=("hip", "torch64"), default="hip")
    args = ap.parse_args()
    from helpers import load_npz, state_dict_torch, Args
    from pcd_reg_hregnet_amd import _lib, train_graph, trainer
    from pcd_reg_hregnet_amd.models import HRegNet
    _lib.load()
    if os.path.exists(os.path.join(REPO, "tests", "golden", args.fixture)):
        fx = load_npz(args.fixture)
    else:  # config 4's rank-0 shard (bench.shard_batch), no reference numbers
        from pcd_reg_hregnet_amd import synthetic
        s, d, Rg, tg = synthetic.lidar_batch(8, 16384, seed0=0)
        nan = np.full((args.steps or 10, 3), np.nan)
        fx = {"src": s, "dst": d, "R_gt": Rg, "t_gt": tg, "lr": np.array(1e-3),
              "loss32": nan, "loss64": nan}
    if args.sim == "torch64":
        train_graph.sim_feats = sim_torch64
    dev = "cuda"
    net = HRegNet(Args())
    net.load_state_dict(state_dict_torch())
    tr = trainer.Trainer(net.to(dev), lr=float(fx["lr"]), alpha=1.0)
    s, d = torch.from_numpy(fx["src"]).to(dev), torch.from_numpy(fx["dst"]).to(dev)
    gR, gt = torch.from_numpy(fx["R_gt"]).to(dev), torch.from_numpy(fx["t_gt"]).to(dev)
    steps = args.steps or fx["loss32"].shape[0]
    ours = [float(tr.step(s, d, gR, gt)[0]) for _ in range(steps)]
    r32, r64 = fx["loss32"][:steps, 0], fx["loss64"][:steps, 0]
    print(json.dumps({"fixture": args.fixture, "sim": args.sim, "ours": [round(x, 6) for x in ours],
                      "ref32": [round(float(x), 6) for x in r32],
                      "ref64": [round(float(x), 6) for x in r64]}), flush=True)


if __name__ == "__main__":
    main()
