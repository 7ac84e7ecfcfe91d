"""CPU oracle for the HRegNet forward hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker (or the timed CPU
baseline).  The product path (``pcd_reg_hregnet_amd``) never imports it.

It is a numpy (float32) restatement of the reference's algorithm, with the
index-exact ops (FPS, WFPS, kNN, gather) in ``hregnet_oracle.c``
(``liboracle.so``, built by ``oracle/Makefile``).  Every function cites the
reference file:line it follows (reference = /root/reference, read as text).

Parity pinning: ``tests/golden/make_golden.py`` ran the reference's own Python
model (``models/HRegNet``) in this container with shims for the unbuilt CUDA
extension (a literal thread-level emulation of ``furthest_point_sampling_gpu.cu``)
and the absent ``pytorch3d`` (brute-force kNN); the fixtures it wrote under
``tests/golden/`` pin this oracle (``tests/test_oracle_golden.py``).
kNN tie order against pytorch3d itself is "parity unpinned" (SURVEY.md 8c).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-C", _HERE, "-s"])
        L = ctypes.CDLL(path)
        f32p = ctypes.POINTER(ctypes.c_float)
        i32p = ctypes.POINTER(ctypes.c_int32)
        L.oracle_opt_n_threads.argtypes = [ctypes.c_int]
        L.oracle_opt_n_threads.restype = ctypes.c_int
        L.oracle_fps.argtypes = [f32p, f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, i32p]
        L.oracle_fps.restype = ctypes.c_int
        L.oracle_fps_temp.argtypes = [f32p, f32p, f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, i32p]
        L.oracle_fps_temp.restype = ctypes.c_int
        L.oracle_knn.argtypes = [f32p, f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, i32p, f32p]
        L.oracle_knn.restype = ctypes.c_int
        L.oracle_gather_points.argtypes = [f32p, i32p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, f32p]
        L.oracle_gather_points_grad.argtypes = [f32p, i32p, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int, ctypes.c_int, f32p]
        L.oracle_num_threads.restype = ctypes.c_int
        L.oracle_nn_radius.argtypes = [f32p, ctypes.c_int, f32p, ctypes.c_int, ctypes.c_float, i32p]
        L.oracle_nn_radius.restype = ctypes.c_int
        _LIB = L
    return _LIB


def _fp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _ip(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


def opt_n_threads(n: int) -> int:
    """cuda_utils.h:22-26"""
    return lib().oracle_opt_n_threads(int(n))


def fps(xyz: np.ndarray, npoint: int, weights: np.ndarray | None = None,
        temp0: np.ndarray | None = None) -> np.ndarray:
    """furthest_point_sampling_gpu.cu:84-206 (weights=None) / :254-375 (weighted).

    xyz [B,N,3] f32, weights [B,N] f32 -> idx [B,npoint] int32.  temp0 [B,N]: the caller's temp
    contents, the kernel's initial running minima (.cu:130); None: 1e10 (models/utils.py:25).
    """
    xyz = np.ascontiguousarray(xyz, dtype=np.float32)
    B, N, _ = xyz.shape
    out = np.zeros((B, npoint), dtype=np.int32)
    w = None
    if weights is not None:
        w = np.ascontiguousarray(weights, dtype=np.float32)
        assert w.shape == (B, N)
    t0 = None if temp0 is None else np.ascontiguousarray(temp0, dtype=np.float32)
    assert t0 is None or t0.shape == (B, N)
    rc = lib().oracle_fps_temp(_fp(xyz), _fp(w) if w is not None else None,
                               _fp(t0) if t0 is not None else None, B, N, npoint, _ip(out))
    assert rc == 0
    return out


def gather_points(points: np.ndarray, idx: np.ndarray) -> np.ndarray:
    """gather_points_kernel_fast (.cu:7-21): [B,C,N] x [B,M] -> [B,C,M]"""
    points = np.ascontiguousarray(points, dtype=np.float32)
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    B, C, N = points.shape
    M = idx.shape[1]
    out = np.empty((B, C, M), dtype=np.float32)
    lib().oracle_gather_points(_fp(points), _ip(idx), B, C, N, M, _fp(out))
    return out


def gather_points_grad(grad_out: np.ndarray, idx: np.ndarray, n: int) -> np.ndarray:
    """gather_points_grad_kernel_fast (.cu:41-55): scatter-add into [B,C,N]."""
    grad_out = np.ascontiguousarray(grad_out, dtype=np.float32)
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    B, C, M = grad_out.shape
    out = np.zeros((B, C, n), dtype=np.float32)
    lib().oracle_gather_points_grad(_fp(grad_out), _ip(idx), B, C, n, M, _fp(out))
    return out


def knn(p1: np.ndarray, p2: np.ndarray, K: int):
    """pytorch3d.ops.knn_points (0.7.8) semantics, canonical (dist, idx) order.

    p1 [B,N1,D], p2 [B,N2,D] -> (dists [B,N1,K] f32, idx [B,N1,K] int64).
    """
    p1 = np.ascontiguousarray(p1, dtype=np.float32)
    p2 = np.ascontiguousarray(p2, dtype=np.float32)
    B, N1, D = p1.shape
    N2 = p2.shape[1]
    idx = np.empty((B, N1, K), dtype=np.int32)
    dist = np.empty((B, N1, K), dtype=np.float32)
    rc = lib().oracle_knn(_fp(p1), _fp(p2), B, N1, N2, D, K, _ip(idx), _fp(dist))
    assert rc == 0
    return dist, idx.astype(np.int64)


def knn_gather(x: np.ndarray, idx: np.ndarray) -> np.ndarray:
    """pytorch3d.ops.knn_gather: x [B,N,C], idx [B,M,K] -> [B,M,K,C]"""
    B = x.shape[0]
    return x[np.arange(B)[:, None, None], idx]


# --------------------------------------------------------------------------
# Layer restatements (models/HRegNet/layers.py), numpy float32, eval-mode BN.
# --------------------------------------------------------------------------
BN_EPS = 1e-5


def _bn(x, sd, pre, axis=1):
    """nn.BatchNorm{1,2}d eval: (x - mean) / sqrt(var + eps) * gamma + beta."""
    shape = [1] * x.ndim
    shape[axis] = -1
    mean = sd[pre + ".running_mean"].reshape(shape)
    var = sd[pre + ".running_var"].reshape(shape)
    g = sd[pre + ".weight"].reshape(shape)
    b = sd[pre + ".bias"].reshape(shape)
    return ((x - mean) / np.sqrt(var + np.float32(BN_EPS)) * g + b).astype(np.float32)


def _conv(x, w, b=None):
    """1x1 Conv{1,2}d over [B,C,...]: y[b,o,...] = sum_c W[o,c] x[b,c,...] (+ bias)."""
    B, C = x.shape[:2]
    rest = x.shape[2:]
    W = w.reshape(w.shape[0], -1)
    y = np.matmul(W[None], x.reshape(B, C, -1)).reshape((B, W.shape[0]) + rest)
    if b is not None:
        y = y + b.reshape((1, -1) + (1,) * len(rest))
    return y.astype(np.float32)


def _conv_stack(x, sd, pre, n):
    """nn.Sequential of n x [Conv(bias=False), BN, ReLU] (layers.py:115-121, 183-189, 246-260)."""
    for i in range(n):
        x = _conv(x, sd[f"{pre}.{3 * i}.weight"])
        x = _bn(x, sd, f"{pre}.{3 * i + 1}")
        x = np.maximum(x, 0)
    return x


def _mlp(x, sd, pre, act=True):
    """Conv1d(bias) [+ BN + ReLU] (layers.py:124-130, 262-268, 425-431)."""
    x = _conv(x, sd[pre + ".0.weight"], sd[pre + ".0.bias"])
    if act:
        x = _bn(x, sd, pre + ".1")
        x = np.maximum(x, 0)
    return x


def _softmax(x, axis=-1):
    m = np.max(x, axis=axis, keepdims=True)
    e = np.exp(x - m)
    return (e / np.sum(e, axis=axis, keepdims=True)).astype(np.float32)


def _softplus(x):
    """nn.Softplus (beta=1, threshold=20)."""
    return np.where(x > 20, x, np.log1p(np.exp(np.minimum(x, 20)))).astype(np.float32)


def _sigmoid(x):
    return (1.0 / (1.0 + np.exp(-x))).astype(np.float32)


def knn_group(xyz1, xyz2, feats2, k):
    """layers.py:9-27: grouped [B,4+C,M,k], knn_xyz [B,M,k,3]."""
    _, idx = knn(xyz1, xyz2, k)
    knn_xyz = knn_gather(xyz2, idx)
    rela = knn_xyz - xyz1[:, :, None, :]
    dist = np.sqrt(np.sum(rela * rela, axis=-1, keepdims=True)).astype(np.float32)
    parts = [rela, dist]
    if feats2 is not None:
        parts.append(knn_gather(np.ascontiguousarray(feats2.transpose(0, 2, 1)), idx))
    g = np.concatenate(parts, axis=-1)
    return np.ascontiguousarray(g.transpose(0, 3, 1, 2)), knn_xyz, idx


def keypoint_detector(sd, pre, xyz, feats, weights, nsample, k, sample=None):
    """KeypointDetector.forward, layers.py:134-165 (fps=True; sample: the random-sampling
    indices [B, nsample] of fps=False, layers.py:144-147)."""
    idx = fps(xyz, nsample, weights) if sample is None else np.asarray(sample, np.int32)
    sampled = gather_points(np.ascontiguousarray(xyz.transpose(0, 2, 1)), idx).transpose(0, 2, 1)
    grouped, knn_xyz, kidx = knn_group(np.ascontiguousarray(sampled), xyz, feats, k)
    emb = _conv_stack(grouped, sd, pre + ".convs", 3)
    x1 = np.max(emb, axis=1)
    a = _softmax(x1, -1)
    keypoints = np.sum(a[..., None] * knn_xyz, axis=2).astype(np.float32)
    att_map = (emb * a[:, None]).astype(np.float32)
    att_feat = np.sum(att_map, axis=-1).astype(np.float32)
    s = _mlp(_mlp(att_feat, sd, pre + ".mlp1"), sd, pre + ".mlp2")
    s = _mlp(s, sd, pre + ".mlp3", act=False)
    sigmas = (_softplus(s) + np.float32(0.001))[:, 0]
    return keypoints, sigmas, att_feat, grouped, att_map, idx, kidx


def desc_extractor(sd, pre, grouped, att_map):
    """DescExtractor.forward, layers.py:200-209."""
    x1 = _conv_stack(grouped, sd, pre + ".convs", 3)
    k = x1.shape[-1]
    x2 = np.repeat(np.max(x1, axis=3, keepdims=True), k, axis=3)
    x2 = np.concatenate([x2, x1, att_map], axis=1)
    x2 = _conv_stack(x2, sd, pre + ".mlp1", 1)
    x2 = _conv_stack(x2, sd, pre + ".mlp2", 1)
    return np.max(x2, axis=3)


def _norm_weights(s):
    """models.py:30-32 / :36-38"""
    w = (np.float32(1.0) / (s + np.float32(1e-5))).astype(np.float32)
    return (w / np.mean(w, axis=1, keepdims=True)).astype(np.float32)


def feature_extraction(sd, points, use_weights=True, samples=None):
    """HierFeatureExtraction.forward, models.py:26-58 (use_fps=True; samples: the three
    levels' random-sampling indices of use_fps=False)."""
    p = "feature_extraction."
    smp = samples if samples is not None else (None, None, None)
    xyz1, s1, f1, g1, m1, i1, k1 = keypoint_detector(sd, p + "detector_1", points, None, None, 1024, 64,
                                                     smp[0])
    d1 = desc_extractor(sd, p + "desc_extractor_1", g1, m1)
    w1 = _norm_weights(s1) if use_weights else None
    xyz2, s2, f2, g2, m2, i2, k2 = keypoint_detector(sd, p + "detector_2", xyz1, f1, w1, 512, 32, smp[1])
    d2 = desc_extractor(sd, p + "desc_extractor_2", g2, m2)
    w2 = _norm_weights(s2) if use_weights else None
    xyz3, s3, f3, g3, m3, i3, k3 = keypoint_detector(sd, p + "detector_3", xyz2, f2, w2, 256, 16, smp[2])
    d3 = desc_extractor(sd, p + "desc_extractor_3", g3, m3)
    return dict(xyz_1=xyz1, xyz_2=xyz2, xyz_3=xyz3, sigmas_1=s1, sigmas_2=s2, sigmas_3=s3,
                desc_1=d1, desc_2=d2, desc_3=d3, fps_idx_1=i1, fps_idx_2=i2, fps_idx_3=i3,
                knn_idx_1=k1, knn_idx_2=k2, knn_idx_3=k3)


def cosine_similarity_matrix(a, b):
    """calc_cosine_similarity (layers.py:29-41) over all pairs:
    S[b,i,j] = <a_i, b_j> / (|a_i| |b_j| + 1e-6); a [B,N,C], b [B,M,C]."""
    ip = np.matmul(a, b.transpose(0, 2, 1))
    na = np.sqrt(np.sum(a * a, axis=-1))
    nb = np.sqrt(np.sum(b * b, axis=-1))
    return (ip / (na[:, :, None] * nb[:, None, :] + np.float32(1e-6))).astype(np.float32)


def _sim_feats(src_d, dst_d, knn_idx):
    """layers.py:292-313 (and :341-362 for the neighbour branch).

    dst_src_cos[b,i,j] = S[b,i,n] / (max_i' S[b,i',n] + 1e-6), n = knn_idx[b,i,j]
    src_dst_cos[b,i,j] = S[b,i,n] / (max_n' S[b,i,n'] + 1e-6)
    where S[b,i,n] = cos(src_i, dst_n).  Returns (src_dst, dst_src) [B,N1,k].
    """
    S = cosine_similarity_matrix(src_d, dst_d)  # [B,N1,N2]
    col_max = np.max(S, axis=1, keepdims=True)  # per dst n (dst_src_cos_max)
    row_max = np.max(S, axis=2, keepdims=True)  # per src i (src_dst_cos_max)
    g = np.take_along_axis(S, knn_idx, axis=2)  # S[b,i,n_ij]
    cm = np.take_along_axis(np.broadcast_to(col_max, S.shape), knn_idx, axis=2)
    src_dst = (g / (row_max + np.float32(1e-6))).astype(np.float32)
    dst_src = (g / (cm + np.float32(1e-6))).astype(np.float32)
    return src_dst, dst_src


def _nbr_desc(sd, pre, xyz, desc, k, rec=None, name=None):
    """neighbour-aware descriptor, layers.py:316-337 (rec[name] = its xyz kNN)."""
    _, idx = knn(xyz, xyz, k)
    knn_xyz = knn_gather(xyz, idx)
    feats = knn_gather(desc, idx)
    rela = knn_xyz - xyz[:, :, None, :]
    dist = np.sqrt(np.sum(rela * rela, axis=-1, keepdims=True)).astype(np.float32)
    f = np.concatenate([feats, rela, dist], axis=-1)
    w = _conv_stack(np.ascontiguousarray(f.transpose(0, 3, 1, 2)), sd, pre + ".convs_2", 3)
    w = _softmax(np.max(w, axis=1), -1)
    if rec is not None:
        rec[name] = idx
    return np.sum(feats * w[..., None], axis=2).astype(np.float32)


def coarse_reg(sd, pre, src_xyz, src_desc, dst_xyz, dst_desc, src_w, dst_w, k=8, rec=None,
               use_sim=True, use_neighbor=True):
    """CoarseReg.forward, layers.py:273-396; rec: the neighbour branch's xyz kNN selections
    (coarse_nbr_src / coarse_nbr_dst).  use_sim / use_neighbor: the constructor's variants
    (layers.py:237-244: convs_1 over 2C + 16 / 14 / 12 inputs; the similarity features
    layers.py:368-379 -- original, neighbour-aware, both or none)."""
    sdsc = np.ascontiguousarray(src_desc.transpose(0, 2, 1))
    ddsc = np.ascontiguousarray(dst_desc.transpose(0, 2, 1))
    _, kidx = knn(sdsc, ddsc, k)
    knn_desc = knn_gather(ddsc, kidx)
    knn_xyz = knn_gather(dst_xyz, kidx)
    xyz_e = np.repeat(src_xyz[:, :, None, :], k, axis=2)
    desc_e = np.repeat(sdsc[:, :, None, :], k, axis=2)
    rela = knn_xyz - xyz_e
    dist = np.sqrt(np.sum(rela * rela, axis=-1, keepdims=True)).astype(np.float32)
    w_e = np.repeat(src_w[:, :, None, None], k, axis=2)
    knn_w = knn_gather(dst_w[..., None], kidx)
    sims = []
    if use_sim:
        sd_cos, ds_cos = _sim_feats(sdsc, ddsc, kidx)
        sims += [sd_cos[..., None], ds_cos[..., None]]
    if use_neighbor:
        snb = _nbr_desc(sd, pre, src_xyz, sdsc, k, rec, "coarse_nbr_src")
        dnb = _nbr_desc(sd, pre, dst_xyz, ddsc, k, rec, "coarse_nbr_dst")
        sd_ncos, ds_ncos = _sim_feats(snb, dnb, kidx)
        sims += [sd_ncos[..., None], ds_ncos[..., None]]
    feats = np.concatenate([rela, dist, xyz_e, knn_xyz, desc_e, knn_desc, w_e, knn_w] + sims, axis=-1)
    f = _conv_stack(np.ascontiguousarray(feats.transpose(0, 3, 1, 2)), sd, pre + ".convs_1", 3)
    a = _softmax(np.max(f, axis=1), -1)
    corres = np.sum(a[..., None] * knn_xyz, axis=2).astype(np.float32)
    att = np.sum(a[:, None] * f, axis=-1).astype(np.float32)
    w = _mlp(_mlp(att, sd, pre + ".mlp1"), sd, pre + ".mlp2")
    w = _mlp(w, sd, pre + ".mlp3", act=False)
    return corres, _sigmoid(w[:, 0]), kidx


def fine_reg(sd, pre, src_xyz, src_feat, dst_xyz, dst_feat, src_w, dst_w, k=8,
             return_att=False):
    """FineReg.forward, layers.py:433-454 (return_att: also the attentive features
    [B, 2C, M] that model_v2/layers.py:471-481 feeds to mlpx)."""
    _, kidx = knn(src_xyz, dst_xyz, k)
    knn_xyz = knn_gather(dst_xyz, kidx)
    sf = np.ascontiguousarray(src_feat.transpose(0, 2, 1))
    df = np.ascontiguousarray(dst_feat.transpose(0, 2, 1))
    knn_f = knn_gather(df, kidx)
    xyz_e = np.repeat(src_xyz[:, :, None, :], k, axis=2)
    f_e = np.repeat(sf[:, :, None, :], k, axis=2)
    rela = knn_xyz - xyz_e
    dist = np.sqrt(np.sum(rela * rela, axis=-1, keepdims=True)).astype(np.float32)
    w_e = np.repeat(src_w[:, :, None, None], k, axis=2)
    knn_w = knn_gather(dst_w[..., None], kidx)
    feats = np.concatenate([rela, dist, xyz_e, knn_xyz, f_e, knn_f, w_e, knn_w], axis=-1)
    f = _conv_stack(np.ascontiguousarray(feats.transpose(0, 3, 1, 2)), sd, pre + ".convs_1", 3)
    a = _softmax(np.max(f, axis=1), -1)
    corres = np.sum(a[..., None] * knn_xyz, axis=2).astype(np.float32)
    att = np.sum(a[:, None] * f, axis=-1).astype(np.float32)
    w = _mlp(_mlp(att, sd, pre + ".mlp1"), sd, pre + ".mlp2")
    w = _mlp(w, sd, pre + ".mlp3", act=False)
    if return_att:
        return corres, _sigmoid(w[:, 0]), kidx, att
    return corres, _sigmoid(w[:, 0]), kidx


def weighted_svd(src, corres, weights):
    """WeightedSVDHead.forward, layers.py:469-504 (fp64 SVD, cast to f32).

    Returns (R [B,3,3], t [B,3]); R = I, t = 0 for the whole batch when the
    SVD cannot run (layers.py:485-493)."""
    eps = 1e-4
    w = weights.astype(np.float64)
    w = w / (np.sum(w, axis=1, keepdims=True) + eps)
    ws = np.sum(w, axis=1)[:, None] + eps
    s = src.astype(np.float64)
    c = corres.astype(np.float64)
    ms = np.einsum("bn,bnd->bd", w, s) / ws
    mc = np.einsum("bn,bnd->bd", w, c) / ws
    sc = s - ms[:, None]
    cc = c - mc[:, None]
    H = np.einsum("bna,bn,bnc->bac", sc, w, cc)
    B = src.shape[0]
    if not np.all(np.isfinite(H)):
        return np.tile(np.eye(3, dtype=np.float32), (B, 1, 1)), np.zeros((B, 3), np.float32)
    U, S, Vt = np.linalg.svd(H)
    V = Vt.transpose(0, 2, 1)
    det = np.linalg.det(np.matmul(V, U.transpose(0, 2, 1)))
    D = np.zeros((B, 3, 3))
    D[:, 0, 0] = 1
    D[:, 1, 1] = 1
    D[:, 2, 2] = det
    R = np.matmul(V, np.matmul(D, U.transpose(0, 2, 1)))
    t = mc - np.einsum("bij,bj->bi", R, ms)
    return R.astype(np.float32), t.astype(np.float32)


def _compose(R_, t_, R, t):
    """T = T_ @ T_prev on 4x4 homogeneous (models.py:100-110, 120-127)."""
    Rn = np.matmul(R_.astype(np.float64), R.astype(np.float64))
    tn = np.einsum("bij,bj->bi", R_.astype(np.float64), t.astype(np.float64)) + t_
    return Rn.astype(np.float32), tn.astype(np.float32)


def _transform(R, t, xyz):
    """R @ xyz^T + t (models.py:91-92, 113-114)."""
    return (np.einsum("bij,bnj->bni", R, xyz) + t[:, None, :]).astype(np.float32)


def hregnet_forward(sd, src, dst, use_weights=True, samples=None):
    """HRegNet.forward, models/HRegNet/models.py:77-148 (eval mode); samples: (src levels
    1-3, dst levels 1-3) random-sampling indices for use_fps=False."""
    sf = feature_extraction(sd, src, use_weights, None if samples is None else samples[:3])
    df = feature_extraction(sd, dst, use_weights, None if samples is None else samples[3:])
    rec = {}
    c3, w3, kd = coarse_reg(sd, "coarse_corres", sf["xyz_3"], sf["desc_3"], df["xyz_3"],
                            df["desc_3"], sf["sigmas_3"], df["sigmas_3"], rec=rec)
    R3, t3 = weighted_svd(sf["xyz_3"], c3, w3)
    x2t = _transform(R3, t3, sf["xyz_2"])
    c2, w2, k2 = fine_reg(sd, "fine_corres_2", x2t, sf["desc_2"], df["xyz_2"], df["desc_2"],
                          sf["sigmas_2"], df["sigmas_2"])
    R2_, t2_ = weighted_svd(x2t, c2, w2)
    R2, t2 = _compose(R2_, t2_, R3, t3)
    x1t = _transform(R2, t2, sf["xyz_1"])
    c1, w1, k1 = fine_reg(sd, "fine_corres_1", x1t, sf["desc_1"], df["xyz_1"], df["desc_1"],
                          sf["sigmas_1"], df["sigmas_1"])
    R1_, t1_ = weighted_svd(x1t, c1, w1)
    R1, t1 = _compose(R1_, t1_, R2, t2)
    # every kNN selection, named as make_golden.py's knn_* fixture keys
    knn_sel = {"coarse_desc_knn": kd, "fine2_knn": k2, "fine1_knn": k1, **rec}
    for lv in (1, 2, 3):
        knn_sel[f"src_knn_{lv}"] = sf[f"knn_idx_{lv}"]
        knn_sel[f"dst_knn_{lv}"] = df[f"knn_idx_{lv}"]
    return dict(src_xyz_corres_3=c3, src_xyz_corres_2=c2, src_xyz_corres_1=c1,
                src_dst_weights_3=w3, src_dst_weights_2=w2, src_dst_weights_1=w1,
                rotation=[R3, R2, R1], translation=[t3, t2, t1], src_feats=sf, dst_feats=df,
                knn_sel=knn_sel)


def model_v2_forward(sd, src, dst, perm_feats, perm_weights, use_weights=True):
    """Model_V2.forward, models/model_v2/models.py:77-183 (eval mode): HRegNet with
    FineReg2 (model_v2/layers.py:462-500), whose attentive features also pass through
    mlpx (Conv1d 2C->C + BN + ReLU).  The "prime" copies are batch-shuffled by the two
    torch.randperm(B) draws the reference makes (features first, then weights,
    models.py:118-119); the caller passes them in."""
    sf = feature_extraction(sd, src, use_weights)
    df = feature_extraction(sd, dst, use_weights)
    rec = {}
    c3, w3, kd = coarse_reg(sd, "coarse_corres", sf["xyz_3"], sf["desc_3"], df["xyz_3"],
                            df["desc_3"], sf["sigmas_3"], df["sigmas_3"], rec=rec)
    R3, t3 = weighted_svd(sf["xyz_3"], c3, w3)
    x2t = _transform(R3, t3, sf["xyz_2"])
    c2, w2, k2, att2 = fine_reg(sd, "fine_corres_2", x2t, sf["desc_2"], df["xyz_2"],
                                df["desc_2"], sf["sigmas_2"], df["sigmas_2"], return_att=True)
    f2 = _mlp(att2, sd, "fine_corres_2.mlpx")
    R2_, t2_ = weighted_svd(x2t, c2, w2)
    R2, t2 = _compose(R2_, t2_, R3, t3)
    x1t = _transform(R2, t2, sf["xyz_1"])
    c1, w1, k1 = fine_reg(sd, "fine_corres_1", x1t, sf["desc_1"], df["xyz_1"], df["desc_1"],
                          sf["sigmas_1"], df["sigmas_1"])
    R1_, t1_ = weighted_svd(x1t, c1, w1)
    R1, t1 = _compose(R1_, t1_, R2, t2)
    knn_sel = {"coarse_desc_knn": kd, "fine2_knn": k2, "fine1_knn": k1, **rec}
    for lv in (1, 2, 3):
        knn_sel[f"src_knn_{lv}"] = sf[f"knn_idx_{lv}"]
        knn_sel[f"dst_knn_{lv}"] = df[f"knn_idx_{lv}"]
    return dict(knn_sel=knn_sel, src_xyz_corres_3=c3, src_xyz_corres_2=c2, src_xyz_corres_1=c1,
                rotation=[R3, R2, R1], translation=[t3, t2, t1],
                src_feats_desc_2=sf["desc_2"], src_feats_sigmas_2=sf["sigmas_2"],
                src_xyz_2_trans=x2t, dst_xyz_2=df["xyz_2"],
                src_dst_feats_2=f2, src_dst_feats_2_prime=f2[np.asarray(perm_feats)],
                src_dst_weights_2=w2, src_dst_weights_2_prime=w2[np.asarray(perm_weights)],
                src_feats=sf, dst_feats=df)


def transformation_loss(pred_R, pred_t, gt_R, gt_t, alpha=1.0):
    """transformation_loss, losses/losses.py:97-164, with pytorch3d 0.7.8's
    matrix_to_euler_angles(E, "XYZ") restated as (atan2(-E12, E22), asin(E02),
    atan2(-E01, E00)) (pytorch3d is absent: SURVEY.md 8c).  fp32 like the reference.
    Returns (loss, loss_R, loss_t, R_err[3], geodesic_dist[B], T_err[3], eucl_dist[B])."""
    f = np.float32
    E = np.matmul(pred_R.transpose(0, 2, 1).astype(f), gt_R.astype(f))
    resi = np.sqrt(np.sum((E - np.eye(3, dtype=f)) ** 2, axis=(1, 2)))
    eul = np.stack([np.arctan2(-E[:, 1, 2], E[:, 2, 2]), np.arcsin(E[:, 0, 2]),
                    np.arctan2(-E[:, 0, 1], E[:, 0, 0])], -1).astype(f)
    R_err = np.mean(np.abs(np.rad2deg(eul)), axis=0)
    cos = np.clip((np.trace(E, axis1=1, axis2=2) - f(1)) / f(2), -1.0, 1.0).astype(f)
    geo = np.rad2deg(np.arccos(cos)).astype(f)
    dt = (pred_t - gt_t).astype(f)
    T_err = np.mean(np.abs(dt), axis=0)
    eucl = np.sqrt(np.sum(dt * dt, axis=1)).astype(f)
    loss_R = np.mean(resi).astype(f)
    loss_t = np.mean(eucl).astype(f)
    return (f(alpha) * loss_R + loss_t, loss_R, loss_t, R_err.astype(f), geo, T_err.astype(f), eucl)


def calib_metrics(pred_tf, gt_tf):
    """CalibEval.add_batch's per-pair numbers (metrics/calibeval.py:72-113) and
    geodesic_distance (:197-214), fp32 like the reference: E = pred_tf @ gt_tf;
    per_pair [B][12] = {deg Euler XYZ of E[:3,:3], E[:3,3], deg Euler XYZ of
    pred_tf[:3,:3], pred_tf[:3,3]}; batch_geo [2] = {mean deg acos((tr-1)/2), mean ||E[:3,3]||}."""
    f = np.float32
    P = np.asarray(pred_tf, f)
    E = np.matmul(P, np.asarray(gt_tf, f)).astype(f)

    def eul(M):
        return np.rad2deg(np.stack([np.arctan2(-M[:, 1, 2], M[:, 2, 2]), np.arcsin(M[:, 0, 2]),
                                    np.arctan2(-M[:, 0, 1], M[:, 0, 0])], -1)).astype(f)

    per = np.concatenate([eul(E[:, :3, :3]), E[:, :3, 3], eul(P[:, :3, :3]), P[:, :3, 3]], 1)
    cos = np.clip((np.trace(E[:, :3, :3], axis1=1, axis2=2) - f(1)) / f(2), -1.0, 1.0).astype(f)
    theta = np.rad2deg(np.arccos(cos)).astype(f)
    tn = np.sqrt(np.sum(E[:, :3, 3] ** 2, axis=1)).astype(f)
    return per.astype(f), np.array([theta.mean(), tn.mean()], f)


# ------------------------------------------- data side
def _sinc(t, kind):
    """sinc1/2/3 with the O(t^8) Taylor branches below 0.01 (transform/rodrigues.py:5-19,
    100-114, 132-145), float32 elementwise."""
    t = np.asarray(t, np.float32)
    t2 = t * t
    small = np.abs(t) < np.float32(0.01)
    with np.errstate(divide="ignore", invalid="ignore"):
        if kind == 1:
            tay = 1 - t2 / 6 * (1 - t2 / 20 * (1 - t2 / 42))
            reg = np.sin(t) / t
        elif kind == 2:
            tay = np.float32(0.5) * (1 - t2 / 12 * (1 - t2 / 30 * (1 - t2 / 56)))
            reg = (1 - np.cos(t)) / t2
        else:
            tay = np.float32(1 / 6) * (1 - t2 / 20 * (1 - t2 / 42 * (1 - t2 / 72)))
            reg = (t - np.sin(t)) / (t * t * t)
    return np.where(small, tay, reg).astype(np.float32)


def _skew(w):
    z = np.zeros_like(w[:, 0])
    return np.stack([np.stack([z, -w[:, 2], w[:, 1]], 1), np.stack([w[:, 2], z, -w[:, 0]], 1),
                     np.stack([-w[:, 1], w[:, 0], z], 1)], 1)


def se3_exp(x):
    """SE3.exp (transform/rodrigues.py:526-553): x [n, 6] -> g [n, 4, 4], float32."""
    x = np.asarray(x, np.float32).reshape(-1, 6)
    w, v = x[:, :3], x[:, 3:]
    t = np.sqrt((w * w).sum(1)).astype(np.float32)[:, None, None]
    W = _skew(w)
    S = W @ W
    eye = np.eye(3, dtype=np.float32)
    R = eye + _sinc(t, 1) * W + _sinc(t, 2) * S
    V = eye + _sinc(t, 2) * W + _sinc(t, 3) * S
    g = np.zeros((len(x), 4, 4), np.float32)
    g[:, :3, :3] = R
    g[:, :3, 3] = (V @ v[:, :, None])[:, :, 0]
    g[:, 3, 3] = 1
    return g


def so3_log(R):
    """SO3.log (transform/rodrigues.py:330-370), including the t = pi branch and the
    NaN-angle case (neither mask: w = 0)."""
    R = np.asarray(R, np.float32)
    tr = (R[:, 0, 0] + R[:, 1, 1]) + R[:, 2, 2]
    with np.errstate(invalid="ignore"):
        t = np.arccos((tr - 1) / 2).astype(np.float32)
    sc = _sinc(t, 1)
    w = np.zeros((len(R), 3), np.float32)
    for i in range(len(R)):
        if abs(sc[i]) > 1e-7:
            d = np.float32(2) * sc[i]
            w[i] = [(R[i, 2, 1] - R[i, 1, 2]) / d, (R[i, 0, 2] - R[i, 2, 0]) / d,
                    (R[i, 1, 0] - R[i, 0, 1]) / d]
        elif abs(sc[i]) <= 1e-7:
            t2 = t[i] * t[i]
            A = (R[i] + np.eye(3, dtype=np.float32)) * t2 / 2
            s3 = np.sign(A[0, 2]) or np.float32(1)
            s23 = np.sign(A[1, 2]) or np.float32(1)
            w[i] = [np.sqrt(A[0, 0]), np.sqrt(A[1, 1]) * (s23 * s3), np.sqrt(A[2, 2]) * s3]
    return w


def se3_log(g):
    """SE3.log (transform/rodrigues.py:571-582, inv_vecs_Xg_ig :400-420)."""
    g = np.asarray(g, np.float32).reshape(-1, 4, 4)
    w = so3_log(g[:, :3, :3])
    t = np.sqrt((w * w).sum(1)).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        t2 = t * t
        eta = np.where(t < 0.01, ((t2 / 40 + 1) * t2 / 42 + 1) * t2 / 720 + np.float32(1 / 12),
                       (1 - (t / 2) / np.tan(t / 2)) / t2).astype(np.float32)
    X = _skew(w)
    H = np.eye(3, dtype=np.float32) - np.float32(0.5) * X + eta[:, None, None] * (X @ X)
    v = (H @ g[:, :3, 3:])[:, :, 0]
    return np.concatenate([w, v], 1).astype(np.float32)


def twists_from_samples(samples, amp_tran, distribution="uniform"):
    """UniformTransformSE3.generate_transform (transform/dataset_transforms.py:79-126)
    from its draws: samples [n, 6] (w draw, t draw), amp_tran [n, 2] float32."""
    s = np.asarray(samples, np.float32)
    amp = np.asarray(amp_tran, np.float32)[:, :1]
    tran = np.asarray(amp_tran, np.float32)[:, 1:]
    if distribution == "uniform":
        w = (2 * s[:, :3] - 1) * amp
        t = (2 * s[:, 3:] - 1) * tran
    else:
        w = s[:, :3] / np.sqrt((s[:, :3] ** 2).sum(1, keepdims=True)) * amp
        u = s[:, 3:] * tran if distribution == "gaussian" else s[:, 3:]
        t = u / np.sqrt((u * u).sum(1, keepdims=True)) * tran
    R = se3_exp(np.concatenate([w, np.zeros_like(w)], 1))
    R[:, :3, 3] = t
    return se3_log(R)


def range_filter(points, intensity, max_range):
    """PointCloudFilter.remove_points_by_range (dataset/dataset_utils.py:113-127)."""
    p = np.asarray(points, np.float32)
    rng = np.sqrt((p[:, 0] * p[:, 0] + p[:, 1] * p[:, 1]) + p[:, 2] * p[:, 2])
    keep = rng < max_range
    return p[keep], (None if intensity is None else np.asarray(intensity)[keep])


def resample_indices(n, num_points):
    """PointCloudResampler.__call__ (dataset/dataset_utils.py:189-223): the rows it keeps,
    drawn from numpy's global RandomState exactly as the reference draws them."""
    if num_points == -1:
        return np.arange(n)
    if n <= num_points:
        return np.concatenate([np.arange(n), np.random.choice(n, num_points - n, replace=True)])
    return np.random.choice(n, num_points, replace=False)


# ------------------------------------- Model_V2 training losses (8f rank 2)
def chamfer_loss(template, source, scale=1.0, reduction="mean"):
    """ChamferDistanceLoss (losses/chamfer_loss.py:10-36) with the chamfer_distance
    extension's nearest squared distances restated (float32, (dx^2+dy^2)+dz^2)."""
    a = np.asarray(template, np.float32) / np.float32(scale)
    b = np.asarray(source, np.float32) / np.float32(scale)
    d = a[:, :, None, :] - b[:, None, :, :]
    dist = (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]
    c01 = np.sqrt(dist.min(2)).mean(-1)
    c10 = np.sqrt(dist.min(1)).mean(-1)
    per = ((c01 + c10) / 2).astype(np.float32)
    return {"none": per, "mean": per.mean(0), "sum": per.sum(0)}[reduction]


def _softplus(z):
    return np.where(z > 20, z, np.log1p(np.exp(np.minimum(z, 20))))


def deep_mi_loss(params, x_global, x_global_prime, x_local, x_local_prime, c_local, c_global):
    """DeepMILoss(512, 128).forward (losses/mi_loss_v2.py:42-79): JS estimator of the
    local ([B, C, N] point rows) and global ([B, C]) discriminators, called as d(c, x)."""
    relu = lambda v: np.maximum(v, 0)  # noqa: E731

    def local_d(c, x):
        h = np.concatenate([c, x], 1).transpose(0, 2, 1)  # [B, N, 2C]
        for k in ("conv1", "conv2", "conv3"):
            h = relu(h @ params[f"local_d.{k}.weight"][:, :, 0].T)
        return h[..., 0]

    def global_d(c, x):
        h = np.concatenate([c, x], 1)
        for k in ("c1", "c2", "c3"):
            h = relu(h @ params[f"global_d.{k}.weight"][:, :, 0].T)
        return h @ params["global_d.l0.weight"].T + params["global_d.l0.bias"]

    def js(d, c, x, xp):
        Ej = -_softplus(-d(c, x)).mean()
        Em = _softplus(d(c, xp)).mean()
        return 0.5 * (Em - Ej)
    loc = js(local_d, c_local, x_local, x_local_prime)
    glo = js(global_d, c_global, x_global, x_global_prime)
    return np.float32(loc + glo), np.float32(loc), np.float32(glo)


def nn_radius(q, p, r):
    """nearest p for each q strictly within r (fp32 distances, ties to the lowest index),
    -1 when none (open3d's hybrid search as registration_icp uses it)"""
    q = np.ascontiguousarray(q, np.float32)
    p = np.ascontiguousarray(p, np.float32)
    out = np.empty(q.shape[0], np.int32)
    lib().oracle_nn_radius(_fp(q), q.shape[0], _fp(p), p.shape[0], np.float32(r) * np.float32(r),
                           _ip(out))
    return out


def _xform64(T, s):
    """p = R s + t in float64, the operation order of csrc/icp.hip xform"""
    s = s.astype(np.float64)
    return np.stack([((T[a, 0] * s[:, 0] + T[a, 1] * s[:, 1]) + T[a, 2] * s[:, 2]) + T[a, 3]
                     for a in range(3)], 1)


def registration_icp(src, dst, max_corr, init=None, rel_fitness=1e-6, rel_rmse=1e-6,
                     max_iteration=30):
    """open3d.pipelines.registration.registration_icp with
    TransformationEstimationPointToPoint (test/test_v4.py:144-158), one pair; open3d is
    not vendored -- its published loop: result_0 = correspondences(T_0); for i <
    max_iteration: T_{i+1} = Kabsch(result_i) T_i, result_{i+1} = correspondences(T_{i+1}),
    stop when fitness and inlier_rmse both move less than the relative criteria.
    Correspondences: nn_radius on the fp32-rounded transformed source (fp64 pose), fitness =
    matches / n_src, inlier_rmse = sqrt(mean d^2) in fp64.  -> (T [4,4] fp64, fitness,
    inlier_rmse, updates applied)."""
    T = np.eye(4) if init is None else np.asarray(init, np.float64).copy()

    def corr(T):
        p64 = _xform64(T, src)
        j = nn_radius(p64.astype(np.float32), dst, max_corr)
        ok = j >= 0
        P, Q = p64[ok], dst[j[ok]].astype(np.float64)
        n = int(ok.sum())
        fit = n / src.shape[0]
        rmse = float(np.sqrt(((P - Q) ** 2).sum() / n)) if n else 0.0
        return P, Q, fit, rmse

    P, Q, fit, rmse = corr(T)
    it = 0
    for it in range(1, max_iteration + 1):
        upd = np.eye(4)
        if P.shape[0]:  # Kabsch (Eigen::umeyama without scaling)
            mp, mq = P.mean(0), Q.mean(0)
            H = (P - mp).T @ (Q - mq)
            U, _, Vt = np.linalg.svd(H)
            V = Vt.T
            D = np.diag([1.0, 1.0, np.sign(np.linalg.det(V @ U.T)) or 1.0])
            R = V @ D @ U.T
            upd[:3, :3], upd[:3, 3] = R, mq - R @ mp
        T = upd @ T
        P, Q, fit2, rmse2 = corr(T)
        conv = abs(fit2 - fit) < rel_fitness and abs(rmse2 - rmse) < rel_rmse
        fit, rmse = fit2, rmse2
        if conv:
            break
    else:
        it = max_iteration
    return T, fit, rmse, it
