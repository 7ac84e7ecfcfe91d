"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Runs in the build container only (the GPU box has no /root/reference).  It
imports the reference's own Python model code (models/HRegNet/*.py,
models/utils.py) unmodified from /root/reference, with shims for what the
container lacks:

* ``point_utils_cuda`` (the unbuilt CUDA extension): a literal numpy
  emulation of furthest_point_sampling_gpu.cu -- bs = opt_n_threads(n)
  virtual threads each keep the FIRST strictly larger d2 over k = t, t+bs, ...
  (.cu:122-134), then the shared-memory tree with __update keeping the lower
  slot on ties (.cu:75-80, 140-199) -- plus gather_points (.cu:7-21).  This is
  written independently of oracle/hregnet_oracle.c so each pins the other.
* ``pytorch3d`` (not installed, no network): knn_points = brute force with the
  distance summed sequentially over d, ordered by (dist, idx); knn_gather =
  indexing.  pytorch3d's own tie order is an unstable sort (parity unpinned).
* ``.cuda()`` -> identity; torch.cuda.IntTensor/FloatTensor -> CPU tensors.

Weights: feature extractor from ckpt/pretrained/nusc_feats.pth
(torch.load(weights_only=True)), saved as tests/golden/nusc_feats.npz; heads
from pcd_reg_hregnet_amd.weights.synthetic_value (trained heads are missing
from the snapshot, .MISSING_LARGE_BLOBS:2-4).

Usage: python tests/golden/make_golden.py [--v2-only | --loss-only | --train-only | --traj-only [--traj-c4] | --ddp-only | --v2-b2-65536 | --forward-only | --v2-train-only | --metrics-only | --perturb-only | --mi-only]   (a few minutes on 8 CPUs)
"""
from __future__ import annotations

import math
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)


# ------------------------------------------------------------------ shims
def opt_n_threads(n: int) -> int:
    p = int(math.log(float(n)) / math.log(2.0))
    return max(min(1 << p, 1024), 1)


def fps_literal(xyz: np.ndarray, m: int, w: np.ndarray | None = None) -> np.ndarray:
    """Thread-level emulation of (weighted_)furthest_point_sampling_kernel, one cloud."""
    n = xyz.shape[0]
    bs = opt_n_threads(n)
    rows = -(-n // bs)
    pad = rows * bs - n
    X = np.concatenate([xyz.astype(np.float32), np.zeros((pad, 3), np.float32)])
    W = None if w is None else np.concatenate([w.astype(np.float32), np.ones(pad, np.float32)])
    valid = np.arange(rows * bs) < n
    temp = np.full(rows * bs, 1e10, np.float32)
    kidx = np.arange(rows * bs).reshape(rows, bs)
    out = np.zeros(m, np.int32)
    old = 0
    for j in range(1, m):
        x1, y1, z1 = X[old]
        dx = X[:, 0] - x1
        dy = X[:, 1] - y1
        dz = X[:, 2] - z1
        d = (dx * dx + dy * dy) + dz * dz
        if W is not None:
            d = W * d
        d2 = np.fmin(d, temp).astype(np.float32)
        temp = np.where(valid, d2, temp)
        d2 = np.where(valid, d2, -np.inf).reshape(rows, bs)
        # per thread: first occurrence of the maximum if it is > -1, else (-1, 0)
        am = np.argmax(d2, axis=0)
        best = d2[am, np.arange(bs)]
        besti = kidx[am, np.arange(bs)]
        ok = best > -1.0
        dists = np.where(ok, best, np.float32(-1.0)).astype(np.float32)
        dists_i = np.where(ok, besti, 0)
        s = bs // 2
        while s >= 1:
            v1, v2 = dists[:s], dists[s:2 * s]
            i1, i2 = dists_i[:s], dists_i[s:2 * s]
            dists_i = np.where(v2 > v1, i2, i1)
            dists = np.maximum(v1, v2)
            s //= 2
        old = int(dists_i[0])
        out[j] = old
    return out


class _PointUtils(types.ModuleType):
    calls: list

    replay: list | None = None

    def _replayed(self, kind, idx):
        if self.replay is None:
            return False
        idx.copy_(self.replay.pop(0))
        self.calls.append((kind, idx.clone()))
        return True

    def furthest_point_sampling_wrapper(self, b, n, m, points, temp, idx):
        if self._replayed("fps", idx):
            return 1
        P = points.detach().cpu().numpy()
        for c in range(b):
            idx[c] = torch.from_numpy(fps_literal(P[c], m))
        self.calls.append(("fps", idx.clone()))
        return 1

    def weighted_furthest_point_sampling_wrapper(self, b, n, m, points, weights, temp, idx):
        if self._replayed("wfps", idx):
            return 1
        P = points.detach().cpu().numpy()
        Wt = weights.detach().cpu().numpy()
        for c in range(b):
            idx[c] = torch.from_numpy(fps_literal(P[c], m, Wt[c]))
        self.calls.append(("wfps", idx.clone()))
        return 1

    def gather_points_wrapper(self, b, c, n, npoints, points, idx, out):
        out.copy_(torch.gather(points, 2, idx.long().unsqueeze(1).expand(b, c, npoints)))
        return 1

    def gather_points_grad_wrapper(self, b, c, n, npoints, grad_out, idx, grad_points):
        grad_points.scatter_add_(2, idx.long().unsqueeze(1).expand(b, c, npoints), grad_out)
        return 1


def knn_brute(p1: torch.Tensor, p2: torch.Tensor, K: int):
    """sum_d (p1_d - p2_d)^2 sequentially over d; stable ascending sort -> (dist, idx)."""
    d = torch.zeros(p1.shape[0], p1.shape[1], p2.shape[1], dtype=torch.float32)
    for e in range(p1.shape[2]):
        diff = p1[:, :, None, e] - p2[:, None, :, e]
        d = d + diff * diff
    dist, idx = torch.sort(d, dim=2, stable=True)
    return dist[:, :, :K].contiguous(), idx[:, :, :K].contiguous()


KNN_CALLS = []
KNN_REPLAY = None  # list of idx tensors to return instead of searching (fp64 replay)


def knn_points(p1, p2, lengths1=None, lengths2=None, norm=2, K=1, version=-1, return_nn=False,
               return_sorted=True):
    if KNN_REPLAY is not None:
        idx = KNN_REPLAY.pop(0)
        dist = None
    else:
        dist, idx = knn_brute(p1.detach().float(), p2.detach().float(), K)
    KNN_CALLS.append(idx.clone())
    nn = knn_gather(p2, idx) if return_nn else None
    return dist, idx, nn


def knn_gather(x, idx, lengths=None):
    B = x.shape[0]
    return x[torch.arange(B)[:, None, None], idx]


def install_shims():
    pu = _PointUtils("point_utils_cuda")
    pu.calls = []
    sys.modules["point_utils_cuda"] = pu
    p3d = types.ModuleType("pytorch3d")
    ops = types.ModuleType("pytorch3d.ops")
    ops.knn_points = knn_points
    ops.knn_gather = knn_gather
    loss = types.ModuleType("pytorch3d.loss")
    loss.chamfer_distance = lambda *a, **k: (_ for _ in ()).throw(NotImplementedError())
    tr = types.ModuleType("pytorch3d.transforms")
    tr.matrix_to_euler_angles = lambda *a, **k: (_ for _ in ()).throw(NotImplementedError())
    p3d.ops, p3d.loss, p3d.transforms = ops, loss, tr
    sys.modules.update({"pytorch3d": p3d, "pytorch3d.ops": ops, "pytorch3d.loss": loss,
                        "pytorch3d.transforms": tr})
    torch.Tensor.cuda = lambda self, *a, **k: self
    torch.nn.Module.cuda = lambda self, *a, **k: self
    torch.cuda.IntTensor = lambda *s: torch.empty(*s, dtype=torch.int32)
    torch.cuda.FloatTensor = lambda *s: torch.empty(*s, dtype=torch.float32)
    # a bare package for /root/reference/models: skips models/__init__.py, which
    # eagerly imports V5/V6 (spconv/flash-attn are absent)
    pkg = types.ModuleType("models")
    pkg.__path__ = [os.path.join(REF, "models")]
    sys.modules["models"] = pkg
    sys.path.insert(0, REF)
    return pu


# ---------------------------------------------------------------- fixtures
def ops_fixtures(rng: np.random.Generator) -> dict:
    out = {}
    # FPS: uniform, tie-heavy (grid-quantised + duplicates), non-power-of-two, m >= n
    cases = []
    x = rng.uniform(-40, 40, (2, 4096, 3)).astype(np.float32)
    cases.append(("uniform4096", x, 512, None))
    g = np.round(rng.uniform(-4, 4, (2, 2048, 3))).astype(np.float32)  # many equal distances
    g[:, 1500:] = g[:, :548]  # exact duplicates
    cases.append(("ties2048", g, 300, None))
    cases.append(("n1000", rng.uniform(-1, 1, (1, 1000, 3)).astype(np.float32), 257, None))
    cases.append(("n100_m100", rng.uniform(-1, 1, (1, 100, 3)).astype(np.float32), 100, None))
    cases.append(("n40_m60", rng.uniform(-1, 1, (1, 40, 3)).astype(np.float32), 60, None))
    cases.append(("l1_16384", rng.uniform(-40, 40, (1, 16384, 3)).astype(np.float32), 1024, None))
    w = rng.uniform(0.2, 3.0, (2, 1024)).astype(np.float32)
    cases.append(("w1024", rng.uniform(-40, 40, (2, 1024, 3)).astype(np.float32), 512, w))
    w2 = np.ones((2, 512), np.float32)
    w2[:, ::3] = 2.0
    cases.append(("wties512", np.round(rng.uniform(-3, 3, (2, 512, 3))).astype(np.float32), 256, w2))
    for name, xyz, m, wt in cases:
        idx = np.stack([fps_literal(xyz[c], m, None if wt is None else wt[c])
                        for c in range(xyz.shape[0])])
        out[f"fps_{name}_xyz"] = xyz
        out[f"fps_{name}_m"] = np.array(m)
        if wt is not None:
            out[f"fps_{name}_w"] = wt
        out[f"fps_{name}_idx"] = idx
    # kNN: xyz K=64 / 8, ties from duplicates, desc-space D=256 K=8, K == n2
    kcases = [
        ("xyz_k64", rng.uniform(-40, 40, (2, 256, 3)), rng.uniform(-40, 40, (2, 4096, 3)), 64),
        ("xyz_ties_k16", np.round(rng.uniform(-3, 3, (1, 128, 3))), np.round(rng.uniform(-3, 3, (1, 700, 3))), 16),
        ("desc_k8", rng.normal(0, 1, (2, 256, 256)), rng.normal(0, 1, (2, 256, 256)), 8),
        ("k_eq_n", rng.uniform(-1, 1, (1, 50, 3)), rng.uniform(-1, 1, (1, 8, 3)), 8),
    ]
    for name, p1, p2, K in kcases:
        p1 = p1.astype(np.float32)
        p2 = p2.astype(np.float32)
        d, i = knn_brute(torch.from_numpy(p1), torch.from_numpy(p2), K)
        out[f"knn_{name}_p1"] = p1
        out[f"knn_{name}_p2"] = p2
        out[f"knn_{name}_dist"] = d.numpy()
        out[f"knn_{name}_idx"] = i.numpy().astype(np.int64)
    return out


class _Args:
    use_fps = True
    use_weights = True
    freeze_detector = False
    freeze_feats = False


class _ArgsRandSample(_Args):
    use_fps = False  # layers.py:144-147 (train_reg_v0.py:52's default: --use_fps is store_true)


def model_fixture(HRegNet, pu, src: np.ndarray, dst: np.ndarray, sd: dict, args=_Args,
                  seed=None) -> dict:
    """The reference's eval forward; with args.use_fps False the random samples are the
    torch.randperm draws after torch.manual_seed(seed), saved as the *_fps_* selections."""
    net = HRegNet(args())
    net.load_state_dict(sd)
    net.eval()
    pu.calls.clear()
    KNN_CALLS.clear()
    draws = []
    randperm = torch.randperm

    def logged(*a, **k):
        r = randperm(*a, **k)
        draws.append(r.clone())
        return r
    if seed is not None:
        torch.manual_seed(seed)
    torch.randperm = logged
    try:
        with torch.no_grad():
            r = net(torch.from_numpy(src), torch.from_numpy(dst))
    finally:
        torch.randperm = randperm
    out = {"src": src, "dst": dst}
    if seed is not None:
        out["perm_seed"] = np.array(seed)
    if not args.use_fps:  # the samples as per-cloud selections (the whole batch shares a draw)
        assert len(draws) == 6, len(draws)
        B = src.shape[0]
        names = ["src_fps_1", "src_fps_2", "src_fps_3", "dst_fps_1", "dst_fps_2", "dst_fps_3"]
        for name, d, m in zip(names, draws, (1024, 512, 256) * 2):
            out[name] = np.broadcast_to(d[:m].numpy().astype(np.int32), (B, m)).copy()
    # the 11 knn_points selections in call order (same sites as the training step's)
    assert len(KNN_CALLS) == len(TRAIN_KNN_NAMES), len(KNN_CALLS)
    for name, idx in zip(TRAIN_KNN_NAMES, KNN_CALLS):
        out["knn_" + name] = idx.numpy().astype(np.int32)
    for i, (R, t) in enumerate(zip(r["rotation"], r["translation"])):
        out[f"R{3 - i}"] = R.numpy()
        out[f"t{3 - i}"] = t.numpy()
    for lv in (1, 2, 3):
        out[f"corres_{lv}"] = r[f"src_xyz_corres_{lv}"].numpy()
        out[f"weights_{lv}"] = r[f"src_dst_weights_{lv}"].numpy()
        for part in ("src", "dst"):
            f = r[f"{part}_feats"]
            out[f"{part}_xyz_{lv}"] = f[f"xyz_{lv}"].numpy()
            out[f"{part}_sigmas_{lv}"] = f[f"sigmas_{lv}"].numpy()
            out[f"{part}_desc_{lv}"] = f[f"desc_{lv}"].numpy()
    # FPS calls in order: src L1, L2, L3, dst L1, L2, L3
    names = ["src_fps_1", "src_fps_2", "src_fps_3", "dst_fps_1", "dst_fps_2", "dst_fps_3"]
    for name, (_, idx) in zip(names, pu.calls):
        out[name] = idx.numpy()
    # the same forward in float64 on the same selections: the fp32 reference's own distance
    # from it is the scale a second fp32 implementation is held to (tests/parity.py)
    r64 = _replay64(HRegNet, pu, sd, src, dst, seed=seed, args=args)
    for i, (R, t) in enumerate(zip(r64["rotation"], r64["translation"])):
        out[f"R{3 - i}_64"] = R.numpy()
        out[f"t{3 - i}_64"] = t.numpy()
    for lv in (1, 2, 3):
        out[f"corres_{lv}_64"] = _f32(r64[f"src_xyz_corres_{lv}"].numpy())
        out[f"weights_{lv}_64"] = _f32(r64[f"src_dst_weights_{lv}"].numpy())
        for part in ("src", "dst"):
            f = r64[f"{part}_feats"]
            for q in ("xyz", "sigmas", "desc"):
                out[f"{part}_{q}_{lv}_64"] = _f32(f[f"{q}_{lv}"].numpy())
    return out


def _f32(x):
    """float64 replay outputs are stored as fp32: the rounding (6e-8 relative) is far below
    every spread and bar they serve (tests/parity.py), at half the fixture size"""
    return np.asarray(x, np.float64).astype(np.float32)


def _replay64(Model, pu, sd, src, dst, seed=None, args=None):
    """The eval forward of `Model` in float64, every FPS / kNN selection replayed from the
    fp32 run just made (pu.calls, KNN_CALLS; random samples: the same seed)."""
    global KNN_REPLAY
    net = Model((args or _Args)())
    net.load_state_dict(sd)
    net = net.double().eval()
    pu.replay = [c[1].clone() for c in pu.calls]
    KNN_REPLAY = [c.clone() for c in KNN_CALLS]
    pu.calls.clear()
    KNN_CALLS.clear()
    torch_eye, torch_zeros = torch.eye, torch.zeros
    torch.eye = lambda *a, **k: torch_eye(*a, **{**k, "dtype": k.get("dtype", torch.float64)})
    torch.zeros = lambda *a, **k: torch_zeros(*a, **{**k, "dtype": k.get("dtype", torch.float64)})
    try:
        if seed is not None:
            torch.manual_seed(seed)
        with torch.no_grad():
            return net(torch.from_numpy(src).double(), torch.from_numpy(dst).double())
    finally:
        torch.eye, torch.zeros = torch_eye, torch_zeros
        pu.replay = None
        KNN_REPLAY = None


def forward_fixtures(HRegNet, pu, sd):
    from pcd_reg_hregnet_amd import synthetic
    # config 1 (BASELINE.json configs[0]): B=1, 2 x 16384 uniform cube, seed 1
    src, dst = synthetic.cube_batch(1, 16384, seed=1)
    np.savez_compressed(os.path.join(HERE, "hregnet_cube_b1_n16384.npz"),
                        **model_fixture(HRegNet, pu, src, dst, sd))
    print("cube fixture written", flush=True)
    # LiDAR-shaped pairs, B=2, N=4096
    s, d, Rg, tg = synthetic.lidar_batch(2, 4096, seed0=0)
    fx = model_fixture(HRegNet, pu, s, d, sd)
    fx["R_gt"], fx["t_gt"] = Rg, tg
    np.savez_compressed(os.path.join(HERE, "hregnet_lidar_b2_n4096.npz"), **fx)
    print("lidar fixture written", flush=True)
    # use_fps=False: random sampling on the seeded host generator (layers.py:144-147)
    fx = model_fixture(HRegNet, pu, s, d, sd, args=_ArgsRandSample, seed=11)
    np.savez_compressed(os.path.join(HERE, "hregnet_randsample_b2_n4096.npz"), **fx)
    print("random-sampling fixture written", flush=True)


def model_v2_fixture(Model_V2, pu, src: np.ndarray, dst: np.ndarray, sd: dict, seed: int) -> dict:
    """Reference Model_V2 forward (models/model_v2/models.py:77-183) in eval mode; the
    randperm "prime" shuffles come from torch's default generator seeded with `seed`."""
    net = Model_V2(_Args())
    net.load_state_dict(sd)
    net.eval()
    pu.calls.clear()
    KNN_CALLS.clear()
    torch.manual_seed(seed)
    with torch.no_grad():
        r = net(torch.from_numpy(src), torch.from_numpy(dst))
    out = {"src": src, "dst": dst, "perm_seed": np.array(seed)}
    assert len(KNN_CALLS) == len(TRAIN_KNN_NAMES), len(KNN_CALLS)
    for name, idx in zip(TRAIN_KNN_NAMES, KNN_CALLS):
        out["knn_" + name] = idx.numpy().astype(np.int32)
    for i, (R, t) in enumerate(zip(r["rotation"], r["translation"])):
        out[f"R{3 - i}"] = R.numpy()
        out[f"t{3 - i}"] = t.numpy()
    for key in ("src_xyz_corres_3", "src_xyz_corres_2", "src_xyz_corres_1", "src_feats_desc_2",
                "src_feats_sigmas_2", "src_xyz_2_trans", "dst_xyz_2", "src_dst_feats_2",
                "src_dst_feats_2_prime", "src_dst_weights_2", "src_dst_weights_2_prime"):
        out[key] = r[key].numpy()
    for lv in (1, 2, 3):
        for part in ("src", "dst"):
            f = r[f"{part}_feats"]
            out[f"{part}_xyz_{lv}"] = f[f"xyz_{lv}"].numpy()
            out[f"{part}_sigmas_{lv}"] = f[f"sigmas_{lv}"].numpy()
            out[f"{part}_desc_{lv}"] = f[f"desc_{lv}"].numpy()
    names = ["src_fps_1", "src_fps_2", "src_fps_3", "dst_fps_1", "dst_fps_2", "dst_fps_3"]
    for name, (_, idx) in zip(names, pu.calls):
        out[name] = idx.numpy()
    r64 = _replay64(Model_V2, pu, sd, src, dst, seed=seed)
    for i, (R, t) in enumerate(zip(r64["rotation"], r64["translation"])):
        out[f"R{3 - i}_64"] = R.numpy()
        out[f"t{3 - i}_64"] = t.numpy()
    for key in ("src_xyz_corres_3", "src_xyz_corres_2", "src_xyz_corres_1", "src_xyz_2_trans",
                "src_dst_feats_2", "src_dst_weights_2"):
        out[key + "_64"] = _f32(r64[key].numpy())
    for lv in (1, 2, 3):
        for part in ("src", "dst"):
            f = r64[f"{part}_feats"]
            for q in ("xyz", "sigmas", "desc"):
                out[f"{part}_{q}_{lv}_64"] = _f32(f[f"{q}_{lv}"].numpy())
    return out


def v2_fixtures_setup():
    """what importing models/model_v2 needs (it takes the helpers from the models package)"""
    import models.utils as mu  # reference helpers, re-exported by models/__init__.py
    pkg = sys.modules["models"]
    for name in ("furthest_point_sample", "weighted_furthest_point_sample", "gather_operation",
                 "set_seed"):
        setattr(pkg, name, getattr(mu, name))
    tr = sys.modules["pytorch3d.transforms"]
    for name in ("axis_angle_to_matrix", "rotation_6d_to_matrix"):
        setattr(tr, name, lambda *a, **k: (_ for _ in ()).throw(NotImplementedError()))


def v2_fixtures(pu):
    """Model_V2 (config 5 shape: 65536-point clouds) fixtures."""
    v2_fixtures_setup()
    from models.model_v2.models import Model_V2  # noqa: E402  (reference code)
    from pcd_reg_hregnet_amd import synthetic, weights
    template = Model_V2(_Args()).state_dict()
    sd = weights.make_state_dict(template, seed=0, pretrained_feats=True)
    s, d, _, _ = synthetic.lidar_batch(2, 4096, seed0=50)
    np.savez_compressed(os.path.join(HERE, "model_v2_lidar_b2_n4096.npz"),
                        **model_v2_fixture(Model_V2, pu, s, d, sd, seed=7))
    print("model_v2 b2 n4096 fixture written", flush=True)
    s, d, _, _ = synthetic.lidar_batch(1, 65536, seed0=60)
    np.savez_compressed(os.path.join(HERE, "model_v2_lidar_b1_n65536.npz"),
                        **model_v2_fixture(Model_V2, pu, s, d, sd, seed=8))
    print("model_v2 b1 n65536 fixture written", flush=True)
    v2_b2_65536_fixture(pu, Model_V2, sd)


def v2_b2_65536_fixture(pu, Model_V2=None, sd=None):
    """config 5's cloud size with two pairs: seed 1 makes both prime
    shuffles (model_v2/layers.py:492,497: torch.randperm(B) for the features, then the
    weights) the swap [1, 0], so the batch permutation is exercised at 65536 points."""
    if Model_V2 is None:
        v2_fixtures_setup()
        from models.model_v2.models import Model_V2  # noqa: E402  (reference code)
        from pcd_reg_hregnet_amd import weights
        sd = weights.make_state_dict(Model_V2(_Args()).state_dict(), seed=0, pretrained_feats=True)
    from pcd_reg_hregnet_amd import synthetic
    torch.manual_seed(1)
    assert torch.randperm(2).tolist() == [1, 0] and torch.randperm(2).tolist() == [1, 0]
    s, d, _, _ = synthetic.lidar_batch(2, 65536, seed0=61)
    np.savez_compressed(os.path.join(HERE, "model_v2_lidar_b2_n65536.npz"),
                        **model_v2_fixture(Model_V2, pu, s, d, sd, seed=1))
    print("model_v2 b2 n65536 fixture written", flush=True)


def p3d_angle_from_tan(axis, other_axis, data, horizontal, tait_bryan):
    """pytorch3d 0.7.8 transforms/rotation_conversions.py _angle_from_tan (restated:
    pytorch3d is not installed here)."""
    i1, i2 = {"X": (2, 1), "Y": (0, 2), "Z": (1, 0)}[axis]
    if horizontal:
        i2, i1 = i1, i2
    even = (axis + other_axis) in ["XY", "YZ", "ZX"]
    if horizontal == even:
        return torch.atan2(data[..., i1], data[..., i2])
    if tait_bryan:
        return torch.atan2(-data[..., i2], data[..., i1])
    return torch.atan2(data[..., i2], -data[..., i1])


def p3d_matrix_to_euler_angles(matrix, convention):
    """pytorch3d 0.7.8 matrix_to_euler_angles (restated; the loss's only pytorch3d call)."""
    idx = {"X": 0, "Y": 1, "Z": 2}
    i0, i2 = idx[convention[0]], idx[convention[2]]
    tait_bryan = i0 != i2
    if tait_bryan:
        central = torch.asin(matrix[..., i0, i2] * (-1.0 if i0 - i2 in [-1, 2] else 1.0))
    else:
        central = torch.acos(matrix[..., i0, i0])
    o = (p3d_angle_from_tan(convention[0], convention[1], matrix[..., i2], False, tait_bryan),
         central,
         p3d_angle_from_tan(convention[2], convention[1], matrix[..., i0, :], True, tait_bryan))
    return torch.stack(o, -1)


def loss_fixtures():
    """Reference transformation_loss (losses/losses.py:97-164) on the HRegNet lidar fixture's
    per-level (R, t) against its ground truth, and on seeded random rotations (small,
    large, and exact-identity errors)."""
    sys.modules["pytorch3d.transforms"].matrix_to_euler_angles = p3d_matrix_to_euler_angles
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_losses", os.path.join(REF, "losses/losses.py"))
    L = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(L)
    from pcd_reg_hregnet_amd import synthetic
    fx = dict(np.load(os.path.join(HERE, "hregnet_lidar_b2_n4096.npz")))
    cases = [(np.stack([fx["R3"], fx["R2"], fx["R1"]]), np.stack([fx["t3"], fx["t2"], fx["t1"]]),
              np.repeat(fx["R_gt"][None], 3, 0), np.repeat(fx["t_gt"][None], 3, 0))]
    rng = np.random.default_rng(77)
    for B, deg in ((16, 2.0), (16, 60.0), (300, 20.0)):
        gR = np.stack([synthetic.random_se3(rng, 180.0)[0] for _ in range(B)]).astype(np.float32)
        dR = np.stack([synthetic.random_se3(rng, deg)[0] for _ in range(B)]).astype(np.float32)
        pR = np.matmul(gR, dR).astype(np.float32)
        if B == 16 and deg == 2.0:
            pR[3] = gR[3]  # exact: geodesic at the acos(1) end
        gt = rng.normal(0, 1, (B, 3)).astype(np.float32)
        pt = (gt + rng.normal(0, 0.1, (B, 3))).astype(np.float32)
        cases.append((pR[None], pt[None], gR[None], gt[None]))
    out = {}
    for c, (pR, pt, gR, gt) in enumerate(cases):
        res = [L.transformation_loss(torch.from_numpy(pR[i]), torch.from_numpy(pt[i]),
                                     torch.from_numpy(gR[i]), torch.from_numpy(gt[i]), alpha=1.5)
               for i in range(pR.shape[0])]
        out[f"c{c}_pred_R"], out[f"c{c}_pred_t"], out[f"c{c}_gt_R"], out[f"c{c}_gt_t"] = pR, pt, gR, gt
        for k, name in enumerate(("loss", "loss_R", "loss_t", "R_err", "geodesic_dist", "T_err",
                                  "eucl_dist")):
            out[f"c{c}_{name}"] = np.stack([r[k].numpy() for r in res])
    out["alpha"] = np.array(1.5, np.float32)
    out["ncases"] = np.array(len(cases))
    np.savez_compressed(os.path.join(HERE, "transformation_loss.npz"), **out)
    print("transformation_loss.npz written", flush=True)


TRAIN_KNN_NAMES = ["src_knn_1", "src_knn_2", "src_knn_3", "dst_knn_1", "dst_knn_2", "dst_knn_3",
                   "coarse_desc_knn", "coarse_nbr_src", "coarse_nbr_dst", "fine2_knn", "fine1_knn"]
TRAIN_FPS_NAMES = ["src_fps_1", "src_fps_2", "src_fps_3", "dst_fps_1", "dst_fps_2", "dst_fps_3"]


FEAT_KEYS = ["xyz_1", "xyz_2", "xyz_3", "sigmas_1", "sigmas_2", "sigmas_3", "desc_1", "desc_2",
             "desc_3"]


def _retain_feats(ret):
    for part in ("src_feats", "dst_feats"):
        for k in FEAT_KEYS:
            ret[part][k].retain_grad()


def _save_feat_grads(ret, out, suffix):
    """gradients of the feature-extraction outputs (models.py:44-56): xyz / sigmas whole,
    desc [B,C,M] as its norm plus the first 64 keypoints of each cloud (float32)"""
    for part in ("src_feats", "dst_feats"):
        for k in FEAT_KEYS:
            g = ret[part][k].grad.detach()
            key = f"fgrad_{part[:3]}_{k}{suffix}"
            out["norm_" + key] = np.array(g.double().norm().item())
            out[key] = (g[:, :, :64] if k.startswith("desc") else g).float().numpy()


def _save_outputs(ret, out, suffix):
    """the train-mode forward's per-level outputs and head results in the tests/parity.py
    fixture layout (so the selections of the train forward are held to the same near-tie
    contract as the eval forward's)"""
    for part in ("src", "dst"):
        f = ret[f"{part}_feats"]
        for lv in (1, 2, 3):
            for q in ("xyz", "sigmas", "desc"):
                out[f"{part}_{q}_{lv}{suffix}"] = _f32(f[f"{q}_{lv}"].detach().numpy())
    for lv in (1, 2, 3):
        out[f"corres_{lv}{suffix}"] = _f32(ret[f"src_xyz_corres_{lv}"].detach().numpy())
        out[f"weights_{lv}{suffix}"] = _f32(ret[f"src_dst_weights_{lv}"].detach().numpy())


def train_fixtures(pu):
    """One reference training step (train/train_reg_v0.py:264-294): HRegNet in .train()
    (batch-statistics BN), l_trans = mean over the 3 levels of transformation_loss
    (alpha 1), loss.backward().  Saved: inputs, every index selection in call order
    (FPS/WFPS, the 11 knn_points calls), per-level R/t, the loss, each parameter's
    gradient (norm, sum, first 256 entries) and every BN running stat after the step."""
    sys.modules["pytorch3d.transforms"].matrix_to_euler_angles = p3d_matrix_to_euler_angles
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_losses", os.path.join(REF, "losses/losses.py"))
    L = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(L)
    from models.HRegNet.models import HRegNet  # noqa: E402  (reference code)
    from pcd_reg_hregnet_amd import synthetic, weights
    template = HRegNet(_Args()).state_dict()
    sd = weights.make_state_dict(template, seed=0, pretrained_feats=True)
    net = HRegNet(_Args())
    net.load_state_dict(sd)
    net.train()
    s, d, Rg, tg = synthetic.lidar_batch(2, 2048, seed0=5)
    pu.calls.clear()
    KNN_CALLS.clear()
    ret = net(torch.from_numpy(s), torch.from_numpy(d))
    _retain_feats(ret)
    gR, gt = torch.from_numpy(Rg), torch.from_numpy(tg)
    l_trans = 0.0
    for i in range(3):
        l_, _, _, _, _, _, _ = L.transformation_loss(ret["rotation"][i], ret["translation"][i], gR,
                                                    gt, 1.0)
        l_trans = l_trans + l_
    loss = l_trans / 3.0
    loss.backward()
    out = {"src": s, "dst": d, "R_gt": Rg, "t_gt": tg, "loss": loss.detach().numpy()}
    for i, (R, t) in enumerate(zip(ret["rotation"], ret["translation"])):
        out[f"R{3 - i}"] = R.detach().numpy()
        out[f"t{3 - i}"] = t.detach().numpy()
    for name, (_, idx) in zip(TRAIN_FPS_NAMES, pu.calls):
        out["idx_" + name] = idx.numpy().astype(np.int32)
    assert len(KNN_CALLS) == len(TRAIN_KNN_NAMES), len(KNN_CALLS)
    for name, idx in zip(TRAIN_KNN_NAMES, KNN_CALLS):
        out["idx_" + name] = idx.numpy().astype(np.int32)
    names = []
    for name, p in net.named_parameters():
        g = p.grad.detach().reshape(-1).double()
        names.append(name)
        out["gnorm_" + name] = np.array(g.norm().item())
        out["gsum_" + name] = np.array(g.sum().item())
        out["ghead_" + name] = g[:256].float().numpy()
    out["param_names"] = np.array(names)
    _save_feat_grads(ret, out, "")
    _save_outputs(ret, out, "")
    for name, b in net.named_buffers():
        if name.endswith("running_mean") or name.endswith("running_var"):
            out["buf_" + name] = b.detach().numpy()
    # the same step in float64 on the same selections: the fp32 reference's own rounding
    # error (|g32 - g64|) is the scale the tests hold our gradients to
    global KNN_REPLAY
    net64 = HRegNet(_Args())
    net64.load_state_dict(sd)
    net64 = net64.double().train()
    pu.replay = [c[1].clone() for c in pu.calls]
    KNN_REPLAY = [c.clone() for c in KNN_CALLS]
    pu.calls.clear()
    KNN_CALLS.clear()
    torch_eye, torch_zeros = torch.eye, torch.zeros
    torch.eye = lambda *a, **k: torch_eye(*a, **{**k, "dtype": k.get("dtype", torch.float64)})
    torch.zeros = lambda *a, **k: torch_zeros(*a, **{**k, "dtype": k.get("dtype", torch.float64)})
    try:
        ret64 = net64(torch.from_numpy(s).double(), torch.from_numpy(d).double())
        _retain_feats(ret64)
        l64 = 0.0
        for i in range(3):
            l64 = l64 + L.transformation_loss(ret64["rotation"][i], ret64["translation"][i],
                                              gR.double(), gt.double(), 1.0)[0]
        (l64 / 3.0).backward()
    finally:
        torch.eye, torch.zeros = torch_eye, torch_zeros
        pu.replay = None
        KNN_REPLAY = None
    out["loss64"] = (l64 / 3.0).detach().numpy()
    _save_feat_grads(ret64, out, "_64")
    _save_outputs(ret64, out, "_64")
    for i, (R, t) in enumerate(zip(ret64["rotation"], ret64["translation"])):
        out[f"R{3 - i}_64"] = R.detach().numpy()
        out[f"t{3 - i}_64"] = t.detach().numpy()
    for name, p in net64.named_parameters():
        g = p.grad.detach().reshape(-1)
        out["g64norm_" + name] = np.array(g.norm().item())
        out["g64head_" + name] = g[:256].numpy()
    np.savez_compressed(os.path.join(HERE, "train_step_b2_n2048.npz"), **out)
    print("train_step_b2_n2048.npz written, loss", float(loss), flush=True)


def _ref_shard_step(HRegNet, L, sd, pu, s, d, Rg, tg):
    """One rank's half of a DDP step (train_reg_v0.py:279-294 on this rank's shard, BN
    statistics of the shard alone): the fp32 train-mode forward + backward and its float64
    replay on the same selections.  -> dict: selections, loss, full fp32 / float64 parameter
    gradients, the BN running stats after the forward."""
    global KNN_REPLAY
    net = HRegNet(_Args())
    net.load_state_dict(sd)
    net.train()
    pu.calls.clear()
    KNN_CALLS.clear()
    ret = net(torch.from_numpy(s), torch.from_numpy(d))
    gR, gt = torch.from_numpy(Rg), torch.from_numpy(tg)
    loss = sum(L.transformation_loss(ret["rotation"][i], ret["translation"][i], gR, gt, 1.0)[0]
               for i in range(3)) / 3.0
    loss.backward()
    out = {"loss": float(loss.detach()), "sel": {}, "g32": {}, "g64": {}, "bufs": {}}
    for name, (_, idx) in zip(TRAIN_FPS_NAMES, pu.calls):
        out["sel"][name] = idx.numpy().astype(np.int32)
    assert len(KNN_CALLS) == len(TRAIN_KNN_NAMES), len(KNN_CALLS)
    for name, idx in zip(TRAIN_KNN_NAMES, KNN_CALLS):
        out["sel"][name] = idx.numpy().astype(np.int32)
    for name, p in net.named_parameters():
        out["g32"][name] = p.grad.detach().reshape(-1).double().numpy()
    for name, b in net.named_buffers():
        if name.endswith("running_mean") or name.endswith("running_var"):
            out["bufs"][name] = b.detach().numpy().copy()
    net64 = HRegNet(_Args())
    net64.load_state_dict(sd)
    net64 = net64.double().train()
    pu.replay = [c[1].clone() for c in pu.calls]
    KNN_REPLAY = [c.clone() for c in KNN_CALLS]
    pu.calls.clear()
    KNN_CALLS.clear()
    torch_eye, torch_zeros = torch.eye, torch.zeros
    torch.eye = lambda *a, **k: torch_eye(*a, **{**k, "dtype": k.get("dtype", torch.float64)})
    torch.zeros = lambda *a, **k: torch_zeros(*a, **{**k, "dtype": k.get("dtype", torch.float64)})
    try:
        r64 = net64(torch.from_numpy(s).double(), torch.from_numpy(d).double())
        l64 = sum(L.transformation_loss(r64["rotation"][i], r64["translation"][i], gR.double(),
                                        gt.double(), 1.0)[0] for i in range(3)) / 3.0
        l64.backward()
    finally:
        torch.eye, torch.zeros = torch_eye, torch_zeros
        pu.replay = None
        KNN_REPLAY = None
    out["loss64"] = float(l64.detach())
    for name, p in net64.named_parameters():
        out["g64"][name] = p.grad.detach().reshape(-1).numpy()
    return out


def ddp_fixtures(pu, B=8, N=2048, seed0=70, ranks=2):
    """SURVEY.md 8(e) / VERDICT r3 item 1: the DDP step of train_reg_v0.py:279-296 over
    `ranks` disjoint shards of one global batch (B / ranks pairs each, rank-local train-mode
    BN as DDP without SyncBN runs it): each rank's gradients, their mean (what the all-reduce
    of DistributedDataParallel hands every rank), each rank's BN running stats, and the
    parameters after torch.optim.Adam(lr=1e-3) applies the mean gradient (identical on every
    rank).  Saved per parameter: norms and the first 256 entries (fp32 and float64 replays)."""
    sys.modules["pytorch3d.transforms"].matrix_to_euler_angles = p3d_matrix_to_euler_angles
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_losses", os.path.join(REF, "losses/losses.py"))
    L = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(L)
    from models.HRegNet.models import HRegNet  # noqa: E402  (reference code)
    from pcd_reg_hregnet_amd import synthetic, weights
    sd = weights.make_state_dict(HRegNet(_Args()).state_dict(), seed=0, pretrained_feats=True)
    s, d, Rg, tg = synthetic.lidar_batch(B, N, seed0=seed0)
    torch.set_num_threads(os.cpu_count())
    out = {"src": s, "dst": d, "R_gt": Rg, "t_gt": tg, "ranks": np.array(ranks),
           "lr": np.array(1e-3)}
    per = B // ranks
    shards = []
    for r in range(ranks):
        sl = slice(r * per, (r + 1) * per)
        sh = _ref_shard_step(HRegNet, L, sd, pu, s[sl], d[sl], Rg[sl], tg[sl])
        shards.append(sh)
        out[f"r{r}_loss"], out[f"r{r}_loss64"] = np.array(sh["loss"]), np.array(sh["loss64"])
        for name, idx in sh["sel"].items():
            out[f"r{r}_idx_{name}"] = idx
        for name, b in sh["bufs"].items():
            out[f"r{r}_buf_{name}"] = b
        for name, g in sh["g32"].items():
            out[f"r{r}_gnorm_{name}"] = np.array(np.linalg.norm(g))
            out[f"r{r}_ghead_{name}"] = g[:256].astype(np.float32)
            g64 = sh["g64"][name]
            out[f"r{r}_g64norm_{name}"] = np.array(np.linalg.norm(g64))
            out[f"r{r}_g64head_{name}"] = g64[:256]
        print(f"rank {r} shard step: loss {sh['loss']:.6f} (float64 {sh['loss64']:.6f})", flush=True)
    names = list(shards[0]["g32"])
    out["param_names"] = np.array(names)
    # the all-reduced gradient: SUM over ranks, then / world (torch DDP's averaging)
    net = HRegNet(_Args())
    net.load_state_dict(sd)
    params = dict(net.named_parameters())
    for name in names:
        g32 = sum(sh["g32"][name].astype(np.float32) for sh in shards) / np.float32(ranks)
        g64 = sum(sh["g64"][name] for sh in shards) / ranks
        out["mean_gnorm_" + name] = np.array(np.linalg.norm(g32.astype(np.float64)))
        out["mean_ghead_" + name] = g32[:256].astype(np.float32)
        out["mean_g64norm_" + name] = np.array(np.linalg.norm(g64))
        out["mean_g64head_" + name] = g64[:256]
        params[name].grad = torch.from_numpy(g32.astype(np.float32)).view_as(params[name])
        out["p0head_" + name] = params[name].detach().reshape(-1)[:256].numpy().copy()
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    opt.step()
    for name in names:
        out["p1head_" + name] = params[name].detach().reshape(-1)[:256].numpy().copy()
    fn = f"ddp_step_r{ranks}_b{B}_n{N}.npz"
    np.savez_compressed(os.path.join(HERE, fn), **out)
    print(fn, "written", flush=True)


def _ref_adam_trajectory(HRegNet, L, sd, s, d, Rg, tg, steps, dtype):
    """`steps` iterations of train_reg_v0.py:279-296 on one fixed batch: zero_grad, the
    train-mode forward, l_trans = mean over the 3 levels of transformation_loss (alpha 1),
    backward, optim.Adam(lr=1e-3) step (train_reg_v0.py:249).  -> per-step loss, l_R, l_t
    (the loss of step i is evaluated before step i's update)."""
    net = HRegNet(_Args())
    net.load_state_dict(sd)
    net = net.to(dtype).train()
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    src, dst = torch.from_numpy(s).to(dtype), torch.from_numpy(d).to(dtype)
    gR, gt = torch.from_numpy(Rg).to(dtype), torch.from_numpy(tg).to(dtype)
    torch_eye, torch_zeros = torch.eye, torch.zeros
    if dtype == torch.float64:
        torch.eye = lambda *a, **k: torch_eye(*a, **{**k, "dtype": k.get("dtype", torch.float64)})
        torch.zeros = lambda *a, **k: torch_zeros(*a, **{**k, "dtype": k.get("dtype", torch.float64)})
    losses = []
    try:
        for _ in range(steps):
            opt.zero_grad()
            ret = net(src, dst)
            lt = lr_ = lt_ = 0.0
            for i in range(3):
                l_, lR, ltr = L.transformation_loss(ret["rotation"][i], ret["translation"][i],
                                                    gR, gt, 1.0)[:3]
                lt, lr_, lt_ = lt + l_, lr_ + lR, lt_ + ltr
            loss = lt / 3.0
            loss.backward()
            opt.step()
            losses.append([float(loss), float(lr_ / 3.0), float(lt_ / 3.0)])
            print(f"  {dtype} step {len(losses)}: loss {losses[-1][0]:.6f}", flush=True)
    finally:
        torch.eye, torch.zeros = torch_eye, torch_zeros
    return np.array(losses, dtype=np.float64)


def trajectory_fixtures(pu, B=2, N=2048, steps=6, seed0=5, name=None):
    """Multi-step reference training trajectory: the reference HRegNet
    trained with torch.optim.Adam on one fixed synthetic batch, in fp32 and in float64
    (both with the shims' selections computed afresh every step).  The fp32-vs-float64
    spread is the scale at which a second fp32 implementation can follow it."""
    sys.modules["pytorch3d.transforms"].matrix_to_euler_angles = p3d_matrix_to_euler_angles
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_losses", os.path.join(REF, "losses/losses.py"))
    L = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(L)
    from models.HRegNet.models import HRegNet  # noqa: E402  (reference code)
    from pcd_reg_hregnet_amd import synthetic, weights
    sd = weights.make_state_dict(HRegNet(_Args()).state_dict(), seed=0, pretrained_feats=True)
    s, d, Rg, tg = synthetic.lidar_batch(B, N, seed0=seed0)
    out = {"R_gt": Rg, "t_gt": tg, "lr": np.array(1e-3), "B": np.array(B), "N": np.array(N),
           "seed0": np.array(seed0), "input_sum": np.array(float(s.astype(np.float64).sum() +
                                                                 d.astype(np.float64).sum()))}
    if B * N <= 8192:  # small: the inputs themselves; config 4: regenerated from the seed
        out.update(src=s, dst=d)
    torch.set_num_threads(os.cpu_count())
    out["loss32"] = _ref_adam_trajectory(HRegNet, L, sd, s, d, Rg, tg, steps, torch.float32)
    out["loss64"] = _ref_adam_trajectory(HRegNet, L, sd, s, d, Rg, tg, steps, torch.float64)
    name = name or f"train_traj_b{B}_n{N}.npz"
    np.savez_compressed(os.path.join(HERE, name), **out)
    print(name, "written:", out["loss32"][:, 0], out["loss64"][:, 0], flush=True)


def v2_train_fixtures(pu):
    """One Model_V2 training step as train/train_reg_v6.py:310-350 takes it: Model_V2 in
    .train() (batch-statistics BN), DeepMILoss(512, 128) (.train()), js_loss = mi(x_global =
    weights_2, x_global_prime, x_local = mlpx features, x_local_prime, c_local = desc_2,
    c_global = sigmas_2) and loss = normalized_c_loss * beta + js_loss * gamma, where the
    Chamfer term is a Python float (c_loss.item()) and so carries no gradient: the gradient
    is js_loss's.  (The script unpacks `ret_dict, corres_dict = net(...)` and reads
    x_global from corres_dict, but model_v2/models.py:183 returns ret_dict alone, whose
    src_dst_weights_2 is the same tensor.)  Saved: inputs, the FPS / kNN selections, the
    two prime draws' seed, js_loss, every parameter gradient (norm, leading entries) of the
    net and the MI loss, and the same step replayed in float64 on the same selections."""
    import importlib.util
    global KNN_REPLAY
    v2_fixtures_setup()
    from models.model_v2.models import Model_V2  # noqa: E402  (reference code)
    from pcd_reg_hregnet_amd import synthetic, weights
    spec = importlib.util.spec_from_file_location("ref_mi_loss_v2", os.path.join(REF, "losses/mi_loss_v2.py"))
    M = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(M)
    sd = weights.make_state_dict(Model_V2(_Args()).state_dict(), seed=0, pretrained_feats=True)
    torch.manual_seed(21)
    mi = M.DeepMILoss(global_in_channels=512, local_in_channels=128)
    mi_sd = {k: v.clone() for k, v in mi.state_dict().items()}
    s, d, _, _ = synthetic.lidar_batch(2, 2048, seed0=5)
    perm_seed = 13
    out = {"src": s, "dst": d, "perm_seed": np.array(perm_seed)}
    out.update({"mi_" + k: v.numpy() for k, v in mi_sd.items()})

    def step(dtype, replay):
        global KNN_REPLAY
        net = Model_V2(_Args())
        net.load_state_dict(sd)
        net = net.to(dtype).train()
        m = M.DeepMILoss(global_in_channels=512, local_in_channels=128)
        m.load_state_dict(mi_sd)
        m = m.to(dtype).train()
        if replay is not None:
            pu.replay = [c.clone() for c in replay[0]]
            KNN_REPLAY = [c.clone() for c in replay[1]]
        pu.calls.clear()
        KNN_CALLS.clear()
        torch_eye, torch_zeros = torch.eye, torch.zeros
        if dtype == torch.float64:
            torch.eye = lambda *a, **k: torch_eye(*a, **{**k, "dtype": k.get("dtype", torch.float64)})
            torch.zeros = lambda *a, **k: torch_zeros(*a, **{**k, "dtype": k.get("dtype", torch.float64)})
        try:
            torch.manual_seed(perm_seed)
            ret = net(torch.from_numpy(s).to(dtype), torch.from_numpy(d).to(dtype))
            js = m(x_global=ret["src_dst_weights_2"], x_global_prime=ret["src_dst_weights_2_prime"],
                   x_local=ret["src_dst_feats_2"], x_local_prime=ret["src_dst_feats_2_prime"],
                   c_local=ret["src_feats"]["desc_2"], c_global=ret["src_feats"]["sigmas_2"])
            js.backward()
        finally:
            torch.eye, torch.zeros = torch_eye, torch_zeros
            pu.replay = None
            KNN_REPLAY = None
        return net, m, js, ret

    net, m, js, ret = step(torch.float32, None)
    sel = ([c[1].clone() for c in pu.calls], [c.clone() for c in KNN_CALLS])
    for name, (_, idx) in zip(TRAIN_FPS_NAMES, pu.calls):
        out["idx_" + name] = idx.numpy().astype(np.int32)
    assert len(KNN_CALLS) == len(TRAIN_KNN_NAMES), len(KNN_CALLS)
    for name, idx in zip(TRAIN_KNN_NAMES, KNN_CALLS):
        out["idx_" + name] = idx.numpy().astype(np.int32)
    out["js"] = js.detach().numpy()
    out["R1"] = ret["rotation"][-1].detach().numpy()
    out["feats_2"] = ret["src_dst_feats_2"].detach().numpy()
    out["weights_2"] = ret["src_dst_weights_2"].detach().numpy()
    names, nograd = [], []
    for prefix, mod in (("net.", net), ("mi.", m)):
        for name, p in mod.named_parameters():
            if p.grad is None:  # outside js_loss's graph (fine_corres_1, ...)
                nograd.append(prefix + name)
                continue
            g = p.grad.detach().reshape(-1).double()
            names.append(prefix + name)
            out["gnorm_" + prefix + name] = np.array(g.norm().item())
            out["ghead_" + prefix + name] = g[:256].float().numpy()
    out["param_names"] = np.array(names)
    out["nograd_names"] = np.array(nograd)
    net64, m64, js64, ret64 = step(torch.float64, sel)
    out["js_64"] = js64.detach().numpy()
    out["feats_2_64"] = ret64["src_dst_feats_2"].detach().numpy()
    for prefix, mod in (("net.", net64), ("mi.", m64)):
        for name, p in mod.named_parameters():
            if p.grad is None:
                continue
            g = p.grad.detach().reshape(-1)
            out["g64norm_" + prefix + name] = np.array(g.norm().item())
            out["g64head_" + prefix + name] = g[:256].numpy()
    np.savez_compressed(os.path.join(HERE, "v2_train_step_b2_n2048.npz"), **out)
    print("v2_train_step_b2_n2048.npz written, js", float(js), float(js64), flush=True)


class _CalibConfig:
    """the attributes CalibEval / MultiLayerCalibEval read (config.py DataConfig)"""
    dataset = "man"

    class dataset_config:
        version = "_v2"
        model = "HRegNet"
        max_trans_error = 0.5
        max_rot_error = 20
        distribution = "uniform"


def metrics_fixtures():
    """The reference's MultiLayerCalibEval (metrics/calibeval.py:340-380) fed as
    test/test_v3.py:130-140 feeds it: 3 levels x 4 batches of 3 pairs; gt_tf = igt (a
    random SE(3) from the synthetic generator), pred_tf = its inverse perturbed by a
    level-dependent small rotation/translation (batch 0, level 2 exactly inverse:
    acos clamp at 1).  Saved: the inputs and results.json as the reference writes it."""
    import importlib.util
    import json
    sys.modules["pytorch3d.transforms"].matrix_to_euler_angles = p3d_matrix_to_euler_angles
    spec = importlib.util.spec_from_file_location("ref_calibeval",
                                                  os.path.join(REF, "metrics/calibeval.py"))
    M = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(M)
    from pcd_reg_hregnet_amd import synthetic
    rng = np.random.default_rng(77)
    ev = M.MultiLayerCalibEval(config=_CalibConfig(), num_layers=3)
    gts, preds = [], []
    for b in range(4):
        _, _, R, t = synthetic.lidar_batch(3, 64, seed0=100 + 3 * b)
        igt = np.tile(np.eye(4, dtype=np.float32), (3, 1, 1))
        igt[:, :3, :3] = R
        igt[:, :3, 3] = t
        inv = np.linalg.inv(igt.astype(np.float64))
        lay = []
        for layer in range(3):
            scale = 0.0 if (b == 0 and layer == 2) else 0.05 / (layer + 1)
            w = rng.normal(0, scale, (3, 3))
            P = inv.copy()
            for i in range(3):
                K = np.array([[0, -w[i, 2], w[i, 1]], [w[i, 2], 0, -w[i, 0]], [-w[i, 1], w[i, 0], 0]])
                th = np.linalg.norm(w[i])
                Rd = np.eye(3) if th == 0 else (np.eye(3) + np.sin(th) / th * K +
                                                (1 - np.cos(th)) / th ** 2 * K @ K)
                P[i, :3, :3] = Rd @ P[i, :3, :3]
                P[i, :3, 3] += rng.normal(0, scale, 3)
            P = P.astype(np.float32)
            lay.append(P)
            ev.add_batch(layer=layer, gt_tf=torch.from_numpy(igt), pred_tf=torch.from_numpy(P))
        gts.append(igt)
        preds.append(np.stack(lay))
    path = os.path.join(HERE, "_calib_results.json")
    ev.save_all_results(path)
    res = open(path).read()
    os.remove(path)
    np.savez_compressed(os.path.join(HERE, "calib_metrics.npz"), gt_tf=np.stack(gts),
                        pred_tf=np.stack(preds), results_json=np.array(res))
    print("calib_metrics.npz written", flush=True)


def perturb_fixtures():
    """The data side in front of the path, from the reference's
    own transform/rodrigues.py, transform/dataset_transforms.py and
    dataset/dataset_utils.py (open3d, imported at its top but unused by the range
    filter and the resampler, is stubbed): SE3 exp/log over small-angle, generic and
    near-pi twists (+ exact pi rotations), UniformTransformSE3 draws per distribution
    under torch.manual_seed, apply_transform, the L2L perturbation + the training
    loop's torch.inverse(igt), the perturbation-file text, the range filter and the
    resampler under np.random.seed."""
    import importlib.util
    pkg = types.ModuleType("transform")
    pkg.__path__ = [os.path.join(REF, "transform")]
    sys.modules["transform"] = pkg
    from transform.rodrigues import SE3, SO3  # noqa: E402  (reference code)
    from transform.dataset_transforms import UniformTransformSE3  # noqa: E402
    sys.modules.setdefault("open3d", types.ModuleType("open3d"))
    spec = importlib.util.spec_from_file_location("ref_dataset_utils",
                                                  os.path.join(REF, "dataset/dataset_utils.py"))
    DU = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(DU)
    from pcd_reg_hregnet_amd import synthetic
    se3, so3 = SE3(), SO3()
    out = {}
    rng = np.random.default_rng(2024)
    axes = rng.normal(size=(96, 3))
    axes /= np.linalg.norm(axes, axis=1, keepdims=True)
    ang = np.concatenate([rng.uniform(1e-5, 9e-3, 16), rng.uniform(0.011, 0.5, 32),
                          rng.uniform(0.5, 3.0, 32), np.pi - rng.uniform(1e-4, 1e-2, 15), [0.0]])
    x = np.concatenate([axes * ang[:, None], rng.normal(0, 0.5, (96, 3))], 1).astype(np.float32)
    xt = torch.from_numpy(x)
    g = se3.exp(xt)
    out["se3_x"] = x
    out["se3_exp"] = g.numpy()
    out["se3_log"] = se3.log(g).numpy()
    # exact pi rotations: the sign-fixed branch of SO3.log (rodrigues.py:347-364)
    pax = np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 1, 0], [0.6, -0.8, 0], [1, 2, -2]],
                   np.float64)
    pax /= np.linalg.norm(pax, axis=1, keepdims=True)
    Rpi = np.stack([2 * np.outer(a, a) - np.eye(3) for a in pax]).astype(np.float32)
    gpi = np.tile(np.eye(4, dtype=np.float32), (len(pax), 1, 1))
    gpi[:, :3, :3] = Rpi
    gpi[:, :3, 3] = rng.normal(0, 0.3, (len(pax), 3))
    out["pi_g"] = gpi
    out["pi_log"] = se3.log(torch.from_numpy(gpi)).numpy()
    # UniformTransformSE3 draws (dataset_config: max_rot_error 20, max_trans_error 0.5)
    for tag, dist, randomly, seed in (("uniform_rand", "uniform", True, 3),
                                      ("uniform_fixed", "uniform", False, 4),
                                      ("gaussian_rand", "gaussian", True, 5),
                                      ("invgauss_rand", "inverse_gaussian", True, 6)):
        torch.manual_seed(seed)
        np.random.seed(seed)
        T = UniformTransformSE3(max_deg=20, max_tran=0.5, distribution=dist, mag_randomly=randomly)
        out[f"twists_{tag}"] = torch.cat([T.generate_transform() for _ in range(24)]).numpy()
    # apply_transform of one cloud [1, 3, N] (a bare [3, N] fails in the reference's
    # SE3.transform: rodrigues.py:589 broadcasts [1,3,3] against [3,N,1])
    s, d, _, _ = synthetic.lidar_batch(4, 2048, seed0=300)
    T = UniformTransformSE3(max_deg=20, max_tran=0.5, mag_randomly=True)
    p0 = torch.from_numpy(d[0].T.copy())[None]
    xa = torch.from_numpy(out["twists_uniform_rand"][:1])
    out["apply_p0"] = p0.numpy()
    out["apply_x"] = xa.numpy()
    out["apply_out"] = T.apply_transform(p0, xa).numpy()
    out["apply_gt"] = T.gt.numpy()
    out["apply_igt"] = T.igt.numpy()
    # L2L batch: man_dataset.py:617-625 per cloud + the loop's torch.inverse(igt)
    xb = torch.from_numpy(out["twists_uniform_rand"][:4])
    unc, igts = [], []
    for b in range(4):
        igt = se3.exp(xb[b:b + 1])
        unc.append(se3.transform(igt, torch.from_numpy(d[b].T.copy())[None]).squeeze(0).T)
        igts.append(igt.squeeze(0))
    out["l2l_pcd"] = d
    out["l2l_x"] = xb.numpy()
    out["l2l_uncalibed"] = torch.stack(unc).numpy()
    out["l2l_igt"] = torch.stack(igts).numpy()
    out["l2l_gt"] = torch.inverse(torch.stack(igts)).numpy()
    # perturbation file text (man_dataset.py:536-545), seed 7, 10 lines
    torch.manual_seed(7)
    T = UniformTransformSE3(max_deg=20, max_tran=0.5, distribution="uniform", mag_randomly=True)
    arr = np.zeros([10, 6])
    for i in range(10):
        arr[i, :] = T.generate_transform().cpu().numpy()
    path = os.path.join(HERE, "_perturb.txt")
    np.savetxt(path, arr, delimiter=",")
    out["perturb_file_text"] = np.array(open(path).read())
    os.remove(path)
    # range filter (max_range 80, dataset/config.json:16) and resampler
    s2, d2, _, _ = synthetic.lidar_batch(1, 8192, seed0=310)
    cloud = np.concatenate([s2[0], d2[0] * 2.2]).astype(np.float32)  # ranges across 80 m
    inten = rng.uniform(0, 1, len(cloud)).astype(np.float32)
    filt = DU.PointCloudFilter(voxel_size=0.01, concat="none", max_range=80)
    fp, fi = filt.remove_points_by_range(cloud, inten)
    out["filter_in"], out["filter_in_int"] = cloud, inten
    out["filter_out"], out["filter_out_int"] = fp, fi
    for tag, n_keep, seed in (("pad", 3000, 11), ("sub", 6000, 12)):
        np.random.seed(seed)
        rs = DU.PointCloudResampler(num_points=4096)
        rp, ri = rs(fp[:n_keep], fi[:n_keep])
        out[f"resample_{tag}_n"] = np.array(n_keep)
        out[f"resample_{tag}_seed"] = np.array(seed)
        out[f"resample_{tag}_out"], out[f"resample_{tag}_int"] = rp, ri
    np.savez_compressed(os.path.join(HERE, "perturb.npz"), **out)
    print("perturb.npz written", flush=True)


def mi_fixtures():
    """Model_V2's training losses from the reference's own
    losses/mi_loss_v2.py (DeepMILoss(512, 128) as train/train_reg_v6.py:253-255 builds
    it, seeded weights, V2-shaped inputs: weights/sigmas [B, 512], feats/desc
    [B, 128, 512]) -- loss and the gradients of every input and parameter -- and
    losses/chamfer_loss.py (ChamferDistanceLoss(scale=50, 'mean'/'none')) over a
    stand-in for the absent third-party chamfer_distance extension: brute-force
    nearest squared distances (its published semantics; the library itself is
    parity-unpinned)."""
    import importlib.util

    class _ChamferDistance(torch.nn.Module):
        def forward(self, a, b):
            d = ((a[:, :, None, :] - b[:, None, :, :]) ** 2).sum(-1)
            d1, i1 = d.min(2)
            d2, i2 = d.min(1)
            return d1, d2, i1, i2
    cd = types.ModuleType("chamfer_distance")
    cd.ChamferDistance = _ChamferDistance
    sys.modules["chamfer_distance"] = cd
    mods = {}
    for name in ("mi_loss_v2", "chamfer_loss"):
        spec = importlib.util.spec_from_file_location("ref_" + name,
                                                      os.path.join(REF, f"losses/{name}.py"))
        mods[name] = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mods[name])
    torch.manual_seed(21)
    mi = mods["mi_loss_v2"].DeepMILoss(global_in_channels=512, local_in_channels=128)
    B = 3
    g = torch.Generator().manual_seed(22)
    inp = {
        "x_global": torch.rand(B, 512, generator=g),                       # weights_2 (sigmoid)
        "x_global_prime": torch.rand(B, 512, generator=g),
        "c_global": torch.rand(B, 512, generator=g) * 2 + 0.01,            # sigmas_2 (softplus)
        "x_local": torch.relu(torch.randn(B, 128, 512, generator=g)),      # mlpx feats (ReLU)
        "x_local_prime": torch.relu(torch.randn(B, 128, 512, generator=g)),
        "c_local": torch.relu(torch.randn(B, 128, 512, generator=g)),      # desc_2 (k-max of ReLU)
    }
    leaves = {k: v.clone().requires_grad_(True) for k, v in inp.items()}
    loss = mi(**leaves)
    loss.backward()
    out = {f"in_{k}": v.numpy() for k, v in inp.items()}
    out.update({f"grad_{k}": v.grad.numpy() for k, v in leaves.items()})
    out.update({f"param_{k}": v.detach().numpy() for k, v in mi.state_dict().items()})
    out.update({f"pgrad_{k}": p.grad.numpy() for k, p in mi.named_parameters()})
    out["loss"] = loss.detach().numpy()
    with torch.no_grad():
        out["loss_local"] = mi.compute_local_loss(inp["x_local"], inp["x_local_prime"],
                                                  inp["c_local"]).numpy()
        out["loss_global"] = mi.compute_global_loss(inp["x_global"], inp["x_global_prime"],
                                                    inp["c_global"]).numpy()
    from pcd_reg_hregnet_amd import synthetic
    s, d, _, _ = synthetic.lidar_batch(3, 512, seed0=500)
    a, b = torch.from_numpy(s), torch.from_numpy(d[:, :400].copy())
    CL = mods["chamfer_loss"].ChamferDistanceLoss
    out["chamfer_a"], out["chamfer_b"] = s, d[:, :400].copy()
    out["chamfer_mean"] = CL(scale=50.0, reduction="mean")(a, b).numpy()
    out["chamfer_none"] = CL(scale=50.0, reduction="none")(a, b).numpy()
    out["chamfer_sum"] = CL(scale=50.0, reduction="sum")(a, b).numpy()
    np.savez_compressed(os.path.join(HERE, "mi_chamfer.npz"), **out)
    print("mi_chamfer.npz written", flush=True)


def main():
    pu = install_shims()
    if "--mi-only" in sys.argv:
        mi_fixtures()
        return
    if "--perturb-only" in sys.argv:
        perturb_fixtures()
        return
    if "--metrics-only" in sys.argv:
        metrics_fixtures()
        return
    if "--train-only" in sys.argv:
        train_fixtures(pu)
        return
    if "--ddp-only" in sys.argv:
        ddp_fixtures(pu)
        return
    if "--traj-only" in sys.argv:
        # B=2 x 2048 pts, 6 steps (test fixture); config 4's shard shape (8 x 16384, the
        # bench's rank-0 batch, seed0 0) with --traj-c4, 14 steps
        if "--traj-c4" in sys.argv:
            trajectory_fixtures(pu, B=8, N=16384, steps=14, seed0=0)
        else:
            trajectory_fixtures(pu)
        return
    if "--v2-train-only" in sys.argv:
        v2_train_fixtures(pu)
        return
    if "--v2-b2-65536" in sys.argv:
        v2_b2_65536_fixture(pu)
        return
    if "--v2-only" in sys.argv:
        v2_fixtures(pu)
        return
    if "--loss-only" in sys.argv:
        loss_fixtures()
        return
    from models.HRegNet.models import HRegNet  # noqa: E402  (reference code)
    from pcd_reg_hregnet_amd import synthetic, weights
    if "--forward-only" in sys.argv:  # the two HRegNet forward fixtures only
        sd = weights.make_state_dict(HRegNet(_Args()).state_dict(), seed=0, pretrained_feats=True)
        forward_fixtures(HRegNet, pu, sd)
        return

    feats = torch.load(os.path.join(REF, "ckpt/pretrained/nusc_feats.pth"), map_location="cpu",
                       weights_only=True)
    np.savez_compressed(os.path.join(HERE, "nusc_feats.npz"),
                        **{k: v.numpy() for k, v in feats.items()})
    template = HRegNet(_Args()).state_dict()
    sd = weights.make_state_dict(template, seed=0, pretrained_feats=True)

    rng = np.random.default_rng(1234)
    np.savez_compressed(os.path.join(HERE, "ops.npz"), **ops_fixtures(rng))
    print("ops.npz written", flush=True)

    forward_fixtures(HRegNet, pu, sd)
    v2_fixtures(pu)
    loss_fixtures()
    train_fixtures(pu)


if __name__ == "__main__":
    main()
