"""How many 64-point blocks a level-1 indexed-kNN query scans (csrc/knn.hip best-first
search, simulated in numpy on a synthetic KITTI-shape cloud) with the spatial index ordered
by the 12-bit Morton cell (counting sort, the order inside a cell left as it comes) or by the
full 30-bit Morton code (HREG_SI_MORTON), and with smaller blocks.

  python tools/knn_block_sim.py [queries]
"""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from pcd_reg_hregnet_amd import synthetic  # noqa: E402

K = 64


def morton(P):
    lo, hi = P.min(0), P.max(0)
    sc = np.where(hi > lo, 1023.99 / (hi - lo), 0)
    q = np.clip(((P - lo) * sc).astype(np.int64), 0, 1023)

    def spread(v):
        out = np.zeros_like(v)
        for b in range(10):
            out |= ((v >> b) & 1) << (3 * b)
        return out
    return spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2)


def visits(P, Q, order, bs):
    S = P[order]
    nb = len(P) // bs
    bmin, bmax = S.reshape(nb, bs, 3).min(1), S.reshape(nb, bs, 3).max(1)
    out = []
    for q in Q:
        lb = (np.maximum(0, np.maximum(bmin - q, q - bmax)) ** 2).sum(1)
        best, tau, v = np.empty(0), np.inf, 0
        for b in np.argsort(lb):
            if lb[b] > tau:
                break
            v += 1
            best = np.sort(np.concatenate([best, ((S[b * bs:(b + 1) * bs] - q) ** 2).sum(1)]))[:K]
            if len(best) == K:
                tau = best[-1]
        out.append(v)
    return np.array(out)


def main():
    nq = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    s, _, _, _ = synthetic.lidar_batch(1, 16384, seed0=3)
    P = s[0].astype(np.float32)
    Q = P[np.random.default_rng(0).choice(len(P), nq, replace=False)]
    code = morton(P)
    for name, order in (("12-bit cell", np.argsort(code >> 18, kind="stable")),
                        ("full Morton", np.argsort(code, kind="stable"))):
        for bs in ((64,) if name.startswith("12") else (64, 32, 16)):
            v = visits(P, Q, order, bs)
            print(f"{name:12s} {bs:2d}-point blocks: {v.mean():5.1f} visited per query (p90 {np.percentile(v, 90):.0f})")


if __name__ == "__main__":
    main()
