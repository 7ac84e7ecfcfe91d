"""Seeded synthetic point-cloud pairs for parity tests and the benchmark.

There is no dataset in this environment, so every
workload is generated here, deterministically per seed, with numpy:

* ``cube_cloud``: ``torch.rand(1, N, 3)``-style uniform cube scaled to
  [-40, 40)^3, the shape of the reference smoke test
  (models/HRegNet/models.py:168-169).
* ``lidar_scan``: a KITTI/MANTruckScenes-shaped scan -- 64 elevation rings in
  [-24.8, +2] deg, ground plane at z = -1.7 m, vertical box structures, range
  <= 80 m (dataset/config.json:16), resampled to N points with duplicate
  padding like PointCloudResampler (dataset/dataset_utils.py:177-223), which
  puts ~2 % duplicate points in (ties for FPS/kNN).
* ``random_se3``: UniformTransformSE3(max_deg=20, max_tran=0.5, 'uniform',
  mag_randomly=True) (transform/dataset_transforms.py:65-126;
  limits dataset/config.json:20-21,24-25).
* ``lidar_pair``: dst = scan, src = R * resample(scan) + t + N(0, 1 cm).
"""
from __future__ import annotations

import numpy as np


def cube_cloud(n: int, rng: np.random.Generator) -> np.ndarray:
    return (rng.random((n, 3), dtype=np.float32) * 80.0 - 40.0).astype(np.float32)


def _rodrigues(w: np.ndarray) -> np.ndarray:
    th = float(np.linalg.norm(w))
    if th < 1e-12:
        return np.eye(3)
    k = w / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * (K @ K)


def random_se3(rng: np.random.Generator, max_deg: float = 20.0, max_tran: float = 0.5):
    """transform/dataset_transforms.py:76-96 ('uniform', mag_randomly=True)."""
    deg = rng.random() * max_deg
    tran = rng.random() * max_tran
    amp = deg * np.pi / 180.0
    w = (2 * rng.random(3) - 1) * amp
    t = (2 * rng.random(3) - 1) * tran
    return _rodrigues(w).astype(np.float64), t.astype(np.float64)


def _raw_scan(rng: np.random.Generator, max_range: float = 80.0) -> np.ndarray:
    """Ring-structured returns from a ground plane plus vertical boxes."""
    n_rings, n_az = 64, 1800
    elev = np.deg2rad(np.linspace(-24.8, 2.0, n_rings))
    az = np.linspace(-np.pi, np.pi, n_az, endpoint=False)
    az = az[None, :] + rng.normal(0, 1e-3, (n_rings, n_az))
    el = elev[:, None] + rng.normal(0, 1e-4, (n_rings, n_az))
    dirs = np.stack([np.cos(el) * np.cos(az), np.cos(el) * np.sin(az), np.sin(el)], -1)
    dirs = dirs.reshape(-1, 3)
    sensor_h = 1.7
    rng_hit = np.full(dirs.shape[0], np.inf)
    down = dirs[:, 2] < -1e-6
    rng_hit[down] = sensor_h / -dirs[down, 2]
    # vertical axis-aligned boxes (cars, walls, poles): slab test per box
    n_boxes = 40
    centers = np.concatenate([rng.uniform(-60, 60, (n_boxes, 2)), np.zeros((n_boxes, 1))], 1)
    half = np.concatenate([rng.uniform(0.3, 6.0, (n_boxes, 2)), rng.uniform(0.5, 4.0, (n_boxes, 1))], 1)
    centers[:, 2] = -sensor_h + half[:, 2]
    inv = 1.0 / np.where(np.abs(dirs) < 1e-9, 1e-9, dirs)
    for c, h in zip(centers, half):
        t0 = (c - h) * inv
        t1 = (c + h) * inv
        tmin = np.max(np.minimum(t0, t1), axis=1)
        tmax = np.min(np.maximum(t0, t1), axis=1)
        hit = (tmax >= np.maximum(tmin, 0)) & (tmin > 0.5)
        rng_hit = np.where(hit & (tmin < rng_hit), tmin, rng_hit)
    ok = np.isfinite(rng_hit) & (rng_hit <= max_range) & (rng_hit > 1.0)
    r = rng_hit[ok] + rng.normal(0, 0.02, ok.sum())
    return (dirs[ok] * r[:, None]).astype(np.float32)


def _resample(pts: np.ndarray, n: int, rng: np.random.Generator, dup_frac: float = 0.02):
    """PointCloudResampler-style: subsample, then pad with duplicates."""
    n_dup = int(round(n * dup_frac))
    n_uniq = min(n - n_dup, pts.shape[0])
    sel = rng.choice(pts.shape[0], n_uniq, replace=False)
    out = pts[sel]
    if out.shape[0] < n:
        extra = out[rng.integers(0, out.shape[0], n - out.shape[0])]
        out = np.concatenate([out, extra], 0)
    perm = rng.permutation(n)
    return np.ascontiguousarray(out[perm]).astype(np.float32)


def lidar_scan(n: int, rng: np.random.Generator) -> np.ndarray:
    return _resample(_raw_scan(rng), n, rng)


def lidar_pair(n: int, seed: int):
    """Returns (src [n,3], dst [n,3], R_gt [3,3], t_gt [3]) with dst ~ R_gt src + t_gt."""
    rng = np.random.default_rng(seed)
    raw = _raw_scan(rng)
    dst = _resample(raw, n, rng)
    src0 = _resample(raw, n, rng)
    R, t = random_se3(rng)
    # src is dst's frame moved by the inverse perturbation: dst = R src + t
    src = ((src0.astype(np.float64) - t) @ R) + rng.normal(0, 0.01, src0.shape)
    return src.astype(np.float32), dst, R.astype(np.float32), t.astype(np.float32)


def lidar_batch(batch: int, n: int, seed0: int = 0):
    """[B,n,3] src/dst batches with seeds seed0 .. seed0+B-1."""
    src, dst, Rs, ts = zip(*(lidar_pair(n, seed0 + b) for b in range(batch)))
    return np.stack(src), np.stack(dst), np.stack(Rs), np.stack(ts)


def cube_batch(batch: int, n: int, seed: int = 1):
    """Config-1 style uniform cubes: src and dst drawn in sequence from one seed."""
    rng = np.random.default_rng(seed)
    src = np.stack([cube_cloud(n, rng) for _ in range(batch)])
    dst = np.stack([cube_cloud(n, rng) for _ in range(batch)])
    return src, dst
