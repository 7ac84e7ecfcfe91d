"""Where does a forward output's error against the reference's float64 replay come from?

Runs the eager forward on a committed fixture with several engine configurations (fused
bf16x6 kernels, fused fp32-MFMA kernels, the layer-by-layer fp32 GEMM path) and prints,
for one output, the normalised error vs float64 of each, of the fp32 reference and of
the CPU oracle, plus the largest-error elements with their values.

  python tools/parity_probe.py [--fixture hregnet_lidar_b2_n4096.npz] [--key dst_desc_3]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

CONFIGS = {
    "bf16x6 fused (product)": {},
    "fp32-MFMA fused": {"B6_L1": False, "B6_L2": False, "B6_L3": False, "B6_HEADS": False,
                        "B6_MLP": False, "B6_GEMM": False},
    "layer-wise fp32 GEMMs": {"FUSED_L1": False, "FUSED_L2": False, "FUSED_L3": False,
                              "B6_GEMM": False, "B6_MLP": False, "FUSED_HEAD": False},
    "no precomputed blocks": {"LEVEL_PRE": False, "HEAD_PRE": False},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fixture", default="hregnet_lidar_b2_n4096.npz")
    ap.add_argument("--key", default="dst_desc_3")
    ap.add_argument("--top", type=int, default=6)
    args = ap.parse_args()
    import parity
    from helpers import Args, load_npz, state_dict_numpy, state_dict_torch
    from oracle import oracle
    from pcd_reg_hregnet_amd import engine
    from pcd_reg_hregnet_amd.models import HRegNet
    g = load_npz(args.fixture)
    B = g["src"].shape[0]
    key = args.key
    ref, ref64 = g[key], g[key + "_64"]
    cm = key.split("_")[1] == "desc"

    def view(x):
        return x.transpose(0, 2, 1) if cm else x

    print(f"{args.fixture} {key}: fp32 reference vs float64 {parity.nerr(view(ref), view(ref64)):.3e}")
    o = parity.as_layout(oracle.hregnet_forward(state_dict_numpy(), g["src"], g["dst"]), B)
    print(f"  CPU oracle (numpy fp32)       vs float64 {parity.nerr(view(o[key]), view(ref64)):.3e}")
    net = HRegNet(Args())
    net.load_state_dict(state_dict_torch())
    net = net.cuda().eval()
    results = {}
    for name, sw in CONFIGS.items():
        saved = {k: getattr(engine, k) for k in sw}
        for k, v in sw.items():
            setattr(engine, k, v)
        try:
            P = engine.PreparedWeights(net.state_dict(), torch.device("cuda"))
            with torch.no_grad():
                r = engine.hregnet_forward(P, torch.from_numpy(g["src"]).cuda(),
                                           torch.from_numpy(g["dst"]).cuda())
            torch.cuda.synchronize()
            cpu = {k2: (v.cpu().numpy() if isinstance(v, torch.Tensor) else v) for k2, v in r.items()}
            for part in ("src_feats", "dst_feats"):
                cpu[part] = {k2: v.cpu().numpy() for k2, v in r[part].items()}
            cpu["rotation"] = [x.cpu().numpy() for x in r["rotation"]]
            cpu["translation"] = [x.cpu().numpy() for x in r["translation"]]
            cpu["_fps_idx"] = [x.cpu().numpy() for x in r["_fps_idx"]]
            lay = parity.as_layout(cpu, B)
        finally:
            for k, v in saved.items():
                setattr(engine, k, v)
        results[name] = lay[key]
        print(f"  {name:28s}  vs float64 {parity.nerr(view(lay[key]), view(ref64)):.3e}"
              f"   vs fp32 ref {parity.nerr(view(lay[key]), view(ref)):.3e}")
    ours = view(results["bf16x6 fused (product)"]).astype(np.float64)
    r64 = view(ref64).astype(np.float64)
    err = np.abs(ours - r64)
    flat = np.argsort(err.reshape(-1))[::-1][:args.top]
    scale = np.abs(r64).max()
    print(f"  largest errors of the product path (scale max|f64| = {scale:.4f}):")
    for f in flat:
        ix = np.unravel_index(f, err.shape)
        vals = "  ".join(f"{n.split()[0]}={view(v)[ix]:.7f}" for n, v in results.items())
        print(f"    {ix}: f64={r64[ix]:.7f} ref32={view(ref)[ix]:.7f} oracle={view(o[key])[ix]:.7f} {vals}")


if __name__ == "__main__":
    main()
