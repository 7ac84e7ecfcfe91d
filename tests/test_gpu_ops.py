"""GPU parity of every C-ABI op against the oracle / reference fixtures.

Index outputs (FPS, kNN) must be bit-exact; float outputs are compared with a
plain fp32 reference (numpy / torch CPU) at the tolerance stated per test.
"""
import numpy as np
import pytest
import torch

from helpers import load_npz
from oracle import oracle

pytestmark = pytest.mark.gpu

OPS = load_npz("ops.npz")
FPS_CASES = sorted({k[4:-4] for k in OPS if k.startswith("fps_") and k.endswith("_idx")})
KNN_CASES = sorted({k[4:-4] for k in OPS if k.startswith("knn_") and k.endswith("_idx")})


def dev(x, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    return t if dtype is None else t.to(dtype)


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from pcd_reg_hregnet_amd import _lib as L
    L.load()
    yield


@pytest.mark.parametrize("case", FPS_CASES)
def test_fps_vs_reference_fixture(case):
    from pcd_reg_hregnet_amd.utils import furthest_point_sample, weighted_furthest_point_sample
    xyz = OPS[f"fps_{case}_xyz"]
    m = int(OPS[f"fps_{case}_m"])
    w = OPS.get(f"fps_{case}_w")
    if w is None:
        got = furthest_point_sample(dev(xyz), m)
    else:
        got = weighted_furthest_point_sample(dev(xyz), dev(w), m)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy(), OPS[f"fps_{case}_idx"])


@pytest.mark.parametrize("n,m,weighted", [(16384, 1024, False), (1024, 512, True), (512, 256, True),
                                          (2048, 700, False), (20000, 64, False), (20000, 64, True),
                                          (3, 5, False), (1, 4, False), (777, 300, True),
                                          (65536, 1024, False), (40000, 300, True),
                                          (131072, 64, False), (140000, 8, False)])
def test_fps_vs_oracle(n, m, weighted):
    from pcd_reg_hregnet_amd import point_utils_cuda as pu
    rng = np.random.default_rng(n * 7 + m)
    B = 3
    xyz = rng.uniform(-40, 40, (B, n, 3)).astype(np.float32)
    xyz[:, n // 2:] = np.round(xyz[:, n // 2:])  # ties
    w = rng.uniform(0.1, 2.0, (B, n)).astype(np.float32) if weighted else None
    idx = torch.empty((B, m), dtype=torch.int32, device="cuda")
    temp = torch.full((B, n), 1e10, device="cuda")
    if weighted:
        pu.weighted_furthest_point_sampling_wrapper(B, n, m, dev(xyz), dev(w), temp, idx)
    else:
        pu.furthest_point_sampling_wrapper(B, n, m, dev(xyz), temp, idx)
    ref = oracle.fps(xyz, m, w)
    np.testing.assert_array_equal(idx.cpu().numpy(), ref)


@pytest.mark.parametrize("n", [16384, 65536, 40000])
@pytest.mark.parametrize("kind", ["lidar", "uniform_ties", "grid_dups", "line"])
def test_fps_indexed_matches_fps(kind, n):
    """hreg_fps_indexed (level-1 FPS over the spatial index's sorted copy, exact pruning:
    fps_sorted_kernel at 16384 points, fps_blocks_kernel above): indices and running minima
    bitwise those of hreg_furthest_point_sampling and the oracle's -- including clouds whose ties
    the reference order must break (rounded coordinates, an integer grid with ~16 copies of every
    point (at 16384), whose last selections are all at T = 0, and a line)."""
    from pcd_reg_hregnet_amd import engine, synthetic, _lib
    m, B = 1024, 3
    rng = np.random.default_rng({"lidar": 1, "uniform_ties": 2, "grid_dups": 3, "line": 4}[kind])
    if kind == "lidar":
        s, d, _, _ = synthetic.lidar_batch(2, n, seed0=12)
        xyz = np.concatenate([s, d])[:B]
    elif kind == "uniform_ties":
        xyz = rng.uniform(-40, 40, (B, n, 3)).astype(np.float32)
        xyz[:, ::2] = np.round(xyz[:, ::2])
    elif kind == "grid_dups":
        xyz = rng.integers(-5, 5, (B, n, 3)).astype(np.float32)
    else:
        t = rng.integers(0, 3000, (B, n)).astype(np.float32)
        xyz = np.stack([t * 0.01, -t * 0.02, np.full_like(t, 3.0)], -1).astype(np.float32)
    xyz = np.ascontiguousarray(xyz, dtype=np.float32)
    x = dev(xyz)
    ws = torch.empty(engine.spatial_index_bytes(B, n), dtype=torch.uint8, device="cuda")
    _lib.call("hreg_spatial_index", x, B, n, ws, _lib.stream_handle())
    idx = torch.full((B, m), -1, dtype=torch.int32, device="cuda")
    temp = torch.full((B, n), -1.0, device="cuda")
    _lib.call("hreg_fps_indexed", B, n, m, x, ws, temp, idx, None, _lib.stream_handle())
    ref = torch.full((B, m), -2, dtype=torch.int32, device="cuda")
    rtemp = torch.full((B, n), 1e10, device="cuda")  # (read: the reference's initial running minima)
    _lib.call("hreg_furthest_point_sampling", B, n, m, x, rtemp, ref, None, _lib.stream_handle())
    torch.cuda.synchronize()
    got = idx.cpu().numpy()
    np.testing.assert_array_equal(got, ref.cpu().numpy())
    if n == 16384:
        assert torch.equal(temp, rtemp)
        # the throughput executor's small-footprint kernel (hreg_fps_indexed_lean,
        # fps_blocks_kernel<4>): the same selections and final running minima
        idx2 = torch.full((B, m), -3, dtype=torch.int32, device="cuda")
        temp2 = torch.full((B, n), -1.0, device="cuda")
        sampled2 = torch.empty(B, m, 3, device="cuda")
        _lib.call("hreg_fps_indexed_lean", B, n, m, x, ws, temp2, idx2, sampled2, _lib.stream_handle())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(idx2.cpu().numpy(), got)
        assert torch.equal(temp2, rtemp)
        np.testing.assert_array_equal(sampled2.cpu().numpy(), xyz[np.arange(B)[:, None], got])
    else:  # (the cluster kernel keeps its exchange slots in temp): the reference's final running
        # minima, min over the centres idx[0 .. m-2] of the two-rounding fp32 distance (.cu:129-130)
        for c in range(B):
            t = np.full(n, 1e10, np.float32)
            p = xyz[c]
            for k in got[c, :-1]:
                d = p - p[k]
                t = np.minimum(t, (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2])
            np.testing.assert_array_equal(temp[c].cpu().numpy(), t)
    np.testing.assert_array_equal(got[:1], oracle.fps(xyz[:1], m, None))


@pytest.mark.parametrize("n", [16384, 65536])
def test_fps_and_indexed_knn_nonfinite_coordinates(n):
    """NaN / inf coordinates: the reference's d2 = fminf(d, temp) (.cu:130)
    keeps temp when d is NaN (a NaN coordinate, inf - inf) or inf, so such a point keeps 1e10 and
    is chosen at the first iteration whose maximum it holds, and from a non-finite centre no
    running minimum moves.  Every GPU FPS path (pruned over the spatial index -- whose Morton key
    maps NaN to cell 0 -- and the register / cluster kernels) must give the oracle's indices; the
    indexed kNN must stay bit-identical to the brute-force scan on the same clouds."""
    from pcd_reg_hregnet_amd import engine, _lib
    from pcd_reg_hregnet_amd import point_utils_cuda as pu
    rng = np.random.default_rng(77 + n)
    B, m = 4, 96
    xyz = rng.uniform(-40, 40, (B, n, 3)).astype(np.float32)
    xyz[:, ::5] = np.round(xyz[:, ::5])
    nanp = rng.integers(1, n, 3)
    xyz[0, nanp[0], 1] = np.nan  # one NaN coordinate
    xyz[1, nanp[1], 0] = np.inf  # +inf
    xyz[1, nanp[2], 2] = -np.inf  # and -inf in the same cloud
    xyz[2, rng.integers(1, n, 40)] = np.nan  # many NaN points
    # cloud 3 stays finite (the pruning must be unaffected beside the others)
    x = dev(xyz)
    ref = oracle.fps(xyz, m, None)
    ws = torch.empty(engine.spatial_index_bytes(B, n), dtype=torch.uint8, device="cuda")
    _lib.call("hreg_spatial_index", x, B, n, ws, _lib.stream_handle())
    a = torch.full((B, m), -1, dtype=torch.int32, device="cuda")
    _lib.call("hreg_fps_indexed", B, n, m, x, ws, None, a, None, _lib.stream_handle())
    b = torch.full((B, m), -2, dtype=torch.int32, device="cuda")
    pu.furthest_point_sampling_wrapper(B, n, m, x, torch.full((B, n), 1e10, device="cuda"), b)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(a.cpu().numpy(), ref)
    np.testing.assert_array_equal(b.cpu().numpy(), ref)
    # the indexed kNN around the selected centres (finite and not) == the brute-force scan
    q = torch.from_numpy(np.ascontiguousarray(xyz[np.arange(B)[:, None], ref])).cuda()
    gi = engine.knn_group_indexed(q, x, 16, ws)
    gb = engine.knn_group(q, x, 16)
    torch.cuda.synchronize()
    assert torch.equal(gi[0], gb[0])


def test_fps_cluster_many_clouds_and_mem_path():
    """n > 16384 runs on the multi-workgroup kernel; more clouds than resident clusters
    (256 / 64 participants = 4) loop; HREG_FPS_MEM forces the single-workgroup
    memory path, which must agree bit for bit."""
    import os
    from pcd_reg_hregnet_amd import point_utils_cuda as pu
    rng = np.random.default_rng(11)
    B, n, m = 20, 65536, 48
    xyz = rng.uniform(-40, 40, (B, n, 3)).astype(np.float32)
    xyz[:, ::3] = np.round(xyz[:, ::3])
    x = dev(xyz)
    a = torch.empty((B, m), dtype=torch.int32, device="cuda")
    b = torch.empty((B, m), dtype=torch.int32, device="cuda")
    pu.furthest_point_sampling_wrapper(B, n, m, x, torch.empty((B, n), device="cuda"), a)
    os.environ["HREG_FPS_MEM"] = "1"
    try:
        pu.furthest_point_sampling_wrapper(B, n, m, x, torch.full((B, n), 1e10, device="cuda"), b)
        torch.cuda.synchronize()
    finally:
        del os.environ["HREG_FPS_MEM"]
    np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())
    np.testing.assert_array_equal(a.cpu().numpy()[:2], oracle.fps(xyz[:2], m, None))


@pytest.mark.parametrize("n,m,weighted", [(16384, 256, False), (1024, 200, True), (700, 100, False)])
def test_fps_reads_callers_temp(n, m, weighted):
    """The caller's temp is the initial running minimum (.cu:130: d2 = min(d, temp[k]); the
    reference's callers fill 1e10, models/utils.py:25, but the boundary's contract is the
    kernel's): random initial minima, some below every distance (those points are never taken),
    against the oracle with the same temp."""
    from pcd_reg_hregnet_amd import point_utils_cuda as pu
    rng = np.random.default_rng(n + m)
    B = 3
    xyz = rng.uniform(-40, 40, (B, n, 3)).astype(np.float32)
    t0 = rng.uniform(0, 3000, (B, n)).astype(np.float32)
    t0[:, ::7] = 1e10
    t0[:, 3::11] = 0.0
    w = rng.uniform(0.1, 2.0, (B, n)).astype(np.float32) if weighted else None
    idx = torch.empty((B, m), dtype=torch.int32, device="cuda")
    temp = dev(t0)
    if weighted:
        pu.weighted_furthest_point_sampling_wrapper(B, n, m, dev(xyz), dev(w), temp, idx)
    else:
        pu.furthest_point_sampling_wrapper(B, n, m, dev(xyz), temp, idx)
    np.testing.assert_array_equal(idx.cpu().numpy(), oracle.fps(xyz, m, w, temp0=t0))


def test_fps_zero_points_requested():
    from pcd_reg_hregnet_amd import point_utils_cuda as pu
    idx = torch.full((2, 1), -7, dtype=torch.int32, device="cuda")
    x = torch.zeros((2, 10, 3), device="cuda")
    pu.furthest_point_sampling_wrapper(2, 10, 0, x, torch.zeros((2, 10), device="cuda"), idx)
    torch.cuda.synchronize()
    assert (idx.cpu() == -7).all()  # m <= 0: kernel returns without writing (.cu:92)


@pytest.mark.parametrize("case", KNN_CASES)
def test_knn_vs_reference_fixture(case):
    from pcd_reg_hregnet_amd.knn import knn_points
    p1, p2 = OPS[f"knn_{case}_p1"], OPS[f"knn_{case}_p2"]
    K = OPS[f"knn_{case}_idx"].shape[-1]
    d, i, nn = knn_points(dev(p1), dev(p2), K=K, return_nn=True)
    np.testing.assert_array_equal(i.cpu().numpy(), OPS[f"knn_{case}_idx"])
    np.testing.assert_array_equal(d.cpu().numpy(), OPS[f"knn_{case}_dist"])
    ref_nn = oracle.knn_gather(p2, OPS[f"knn_{case}_idx"])
    np.testing.assert_array_equal(nn.cpu().numpy(), ref_nn)


@pytest.mark.parametrize("n1,n2,dim,K", [(1024, 16384, 3, 64), (512, 1024, 3, 32), (256, 512, 3, 16),
                                         (256, 256, 256, 8), (33, 70, 5, 8), (10, 5, 3, 8),
                                         (37, 200, 64, 8), (100, 300, 128, 16), (3, 6, 8, 8)])
def test_knn_vs_oracle(n1, n2, dim, K):
    from pcd_reg_hregnet_amd.knn import knn_points
    rng = np.random.default_rng(n1 + n2 + dim + K)
    p1 = rng.normal(size=(2, n1, dim)).astype(np.float32)
    p2 = rng.normal(size=(2, n2, dim)).astype(np.float32)
    p2[:, n2 // 2:] = p2[:, : n2 - n2 // 2]  # duplicate points -> distance ties
    d, i, _ = knn_points(dev(p1), dev(p2), K=K)
    rd, ri = oracle.knn(p1, p2, K)
    np.testing.assert_array_equal(i.cpu().numpy(), ri)
    np.testing.assert_array_equal(d.cpu().numpy(), rd)


def test_knn_group_matches_oracle():
    from pcd_reg_hregnet_amd import engine
    rng = np.random.default_rng(5)
    nb, n, m, k = 3, 4096, 256, 64
    p = rng.uniform(-40, 40, (nb, n, 3)).astype(np.float32)
    q = p[:, rng.choice(n, m, replace=False)]
    gidx, geom, kx = engine.knn_group(dev(q), dev(p), k)
    _, ri = oracle.knn(q, p, k)
    glob = (ri + (np.arange(nb) * n)[:, None, None]).reshape(-1)
    np.testing.assert_array_equal(gidx.cpu().numpy(), glob)
    nnp = oracle.knn_gather(p, ri).reshape(-1, 3)
    np.testing.assert_array_equal(kx.cpu().numpy(), nnp)
    rela = nnp - np.repeat(q.reshape(-1, 3), k, 0)
    np.testing.assert_array_equal(geom.cpu().numpy()[:, :3], rela)
    np.testing.assert_allclose(geom.cpu().numpy()[:, 3], np.linalg.norm(rela, axis=-1), rtol=1e-6)


def test_gather_points_and_grad():
    from pcd_reg_hregnet_amd.utils import gather_operation
    rng = np.random.default_rng(1)
    feats = rng.normal(size=(2, 3, 1000)).astype(np.float32)
    idx = rng.integers(0, 1000, (2, 300)).astype(np.int32)
    f = dev(feats).requires_grad_(True)
    out = gather_operation(f, dev(idx))
    np.testing.assert_array_equal(out.detach().cpu().numpy(), oracle.gather_points(feats, idx))
    go = rng.normal(size=(2, 3, 300)).astype(np.float32)
    out.backward(dev(go))
    np.testing.assert_allclose(f.grad.cpu().numpy(), oracle.gather_points_grad(go, idx, 1000),
                               rtol=1e-6, atol=1e-6)


def test_knn_gather_and_grad():
    from pcd_reg_hregnet_amd.knn import knn_gather
    rng = np.random.default_rng(2)
    x = rng.normal(size=(2, 50, 7)).astype(np.float32)
    idx = rng.integers(0, 50, (2, 20, 4)).astype(np.int64)
    xt = dev(x).requires_grad_(True)
    out = knn_gather(xt, dev(idx))
    np.testing.assert_array_equal(out.detach().cpu().numpy(), oracle.knn_gather(x, idx))
    out.sum().backward()
    cnt = np.zeros((2, 50))
    for b in range(2):
        np.add.at(cnt[b], idx[b].reshape(-1), 1)
    np.testing.assert_allclose(xt.grad.cpu().numpy(), np.repeat(cnt[..., None], 7, -1), rtol=1e-6)
    # random gradients, padded (-1) entries: the CSR scatter sums in ascending (m, k) order --
    # the fp32 serial sum, bitwise -- and is deterministic run to run (no atomics)
    idx[0, 3, 2] = -1
    idx[1, 7, :] = -1
    go = rng.normal(size=(2, 20, 4, 7)).astype(np.float32)
    grads = []
    for _ in range(2):
        xt.grad = None
        knn_gather(xt, dev(idx)).backward(dev(go))
        grads.append(xt.grad.cpu().numpy())
    want = np.zeros((2, 50, 7), np.float32)
    for b in range(2):
        for m in range(20):
            for k in range(4):
                if idx[b, m, k] >= 0:
                    want[b, idx[b, m, k]] += go[b, m, k]
    np.testing.assert_array_equal(grads[0], want)
    np.testing.assert_array_equal(grads[1], grads[0])


@pytest.mark.parametrize("R,N,segs", [
    (1000, 32, [(4, "plain")]),
    (4096, 64, [(4, "plain"), (64, "gather")]),
    (3000, 128, [(128, "div"), (128, "plain"), (256, "scale")]),
    (2048, 512, [(16, "plain"), (256, "div"), (256, "gather")]),
    (777, 96, [(12, "plain"), (64, "gather")]),
    (16384, 512, [(512, "plain")]),
    (1000, 200, [(36, "plain"), (100, "gather")]),
])
@pytest.mark.parametrize("b6", [False, True])
def test_gemm_segments_vs_torch_fp32(R, N, segs, b6):
    """fp32 MFMA GEMM (b6: hreg_gemm6, bf16x6 products on the bf16 matrix cores) with
    gathered/repeated/scaled segments vs torch fp32 on CPU.  Tolerance: 1e-5 relative to
    sum|a*w| (fp32 accumulation-order differences) for both."""
    from pcd_reg_hregnet_amd import engine
    rng = np.random.default_rng(R + N)
    K = sum(c for c, _ in segs)
    W = (rng.normal(size=(N, K)) / np.sqrt(K)).astype(np.float32)
    alpha = rng.uniform(0.5, 1.5, N).astype(np.float32)
    beta = rng.normal(0, 0.1, N).astype(np.float32)
    lin = engine.Lin(dev(W), dev(alpha), dev(beta), True)
    parts, dsegs, keep = [], [], []
    k0 = 0
    k = 8
    for c, kind in segs:
        if kind == "plain":
            src = rng.normal(size=(R, c)).astype(np.float32)
            parts.append(src)
            t = dev(src); keep.append(t)
            dsegs.append(engine._seg(t, k0, c))
        elif kind == "gather":
            src = rng.normal(size=(500, c)).astype(np.float32)
            gi = rng.integers(0, 500, R).astype(np.int32)
            parts.append(src[gi])
            t, tg = dev(src), dev(gi); keep += [t, tg]
            dsegs.append(engine._seg(t, k0, c, gather=tg))
        elif kind == "div":
            src = rng.normal(size=((R + k - 1) // k, c)).astype(np.float32)
            parts.append(src[np.arange(R) // k])
            t = dev(src); keep.append(t)
            dsegs.append(engine._seg(t, k0, c, row_div=k))
        else:
            src = rng.normal(size=(R, c)).astype(np.float32)
            sc = rng.uniform(0, 1, R).astype(np.float32)
            parts.append((src * sc[:, None]).astype(np.float32))
            t, ts = dev(src), dev(sc); keep += [t, ts]
            dsegs.append(engine._seg(t, k0, c, rowscale=ts))
        k0 += c
    A = np.concatenate(parts, 1)
    out = engine.gemm(dsegs, lin, R, b6=b6).cpu().numpy()
    ref = torch.from_numpy(A) @ torch.from_numpy(W).T
    ref = torch.relu(ref * torch.from_numpy(alpha) + torch.from_numpy(beta)).numpy()
    scale = (np.abs(A) @ np.abs(W).T) * alpha + np.abs(beta)
    assert np.all(np.abs(out - ref) <= 1e-5 * scale + 1e-6)


def test_cosine_gemm_vs_torch():
    from pcd_reg_hregnet_amd import engine
    rng = np.random.default_rng(3)
    B, n1, n2, C = 3, 256, 256, 256
    a = rng.normal(size=(B * n1, C)).astype(np.float32)
    b = rng.normal(size=(B * n2, C)).astype(np.float32)
    S = torch.empty((B, n1, n2), device="cuda")
    ta, tb = dev(a), dev(b)
    na, nb = engine.row_norms(ta), engine.row_norms(tb)
    engine.cosine_gemm(ta, tb, na, nb, B, n1, n2, C, S)
    ref = oracle.cosine_similarity_matrix(a.reshape(B, n1, C), b.reshape(B, n2, C))
    np.testing.assert_allclose(S.cpu().numpy(), ref, rtol=1e-5, atol=1e-6)


def test_attend_and_group_max_vs_numpy():
    from pcd_reg_hregnet_amd import engine
    rng = np.random.default_rng(4)
    G, k, C = 300, 32, 128
    emb = np.maximum(rng.normal(size=(G * k, C)), 0).astype(np.float32)
    xyz = rng.normal(size=(G * k, 3)).astype(np.float32)
    attw, att, kp = engine.attend(dev(emb), G, k, vals=dev(emb), xyz_rows=dev(xyz), want_attw=True)
    x1 = emb.reshape(G, k, C).max(-1)
    a = oracle._softmax(x1, -1)
    np.testing.assert_allclose(attw.cpu().numpy().reshape(G, k), a, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(kp.cpu().numpy(), (a[..., None] * xyz.reshape(G, k, 3)).sum(1),
                               rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(att.cpu().numpy(), (emb.reshape(G, k, C) * a[..., None]).sum(1),
                               rtol=1e-5, atol=1e-6)
    gm = engine.group_max(dev(emb), G, k)
    np.testing.assert_array_equal(gm.cpu().numpy(), emb.reshape(G, k, C).max(1))


def test_weighted_svd_recovers_planted_transform():
    """Known answer: corres = R s + t exactly -> (R, t) recovered."""
    from pcd_reg_hregnet_amd import engine, synthetic
    rng = np.random.default_rng(6)
    B, n = 5, 1024
    src = rng.uniform(-20, 20, (B, n, 3)).astype(np.float32)
    Rs, ts = zip(*(synthetic.random_se3(rng) for _ in range(B)))
    Rs, ts = np.stack(Rs).astype(np.float32), np.stack(ts).astype(np.float32)
    cor = (np.einsum("bij,bnj->bni", Rs, src) + ts[:, None]).astype(np.float32)
    w = rng.uniform(0.1, 1.0, (B, n)).astype(np.float32)
    _, _, R, t = engine.weighted_svd(dev(src), dev(cor), dev(w))
    np.testing.assert_allclose(R.cpu().numpy(), Rs, atol=2e-5)
    np.testing.assert_allclose(t.cpu().numpy(), ts, atol=2e-4)
    oR, ot = oracle.weighted_svd(src, cor, w)
    np.testing.assert_allclose(R.cpu().numpy(), oR, atol=1e-5)
    np.testing.assert_allclose(t.cpu().numpy(), ot, atol=1e-4)


def test_weighted_svd_nonfinite_batch_fallback():
    """layers.py:485-493: a failing SVD gives R = I, t = 0 for the whole batch."""
    from pcd_reg_hregnet_amd import engine
    rng = np.random.default_rng(7)
    src = rng.normal(size=(3, 64, 3)).astype(np.float32)
    cor = src.copy()
    cor[1, 5, 0] = np.nan
    w = np.ones((3, 64), np.float32)
    _, _, R, t = engine.weighted_svd(dev(src), dev(cor), dev(w))
    np.testing.assert_array_equal(R.cpu().numpy(), np.tile(np.eye(3, dtype=np.float32), (3, 1, 1)))
    np.testing.assert_array_equal(t.cpu().numpy(), np.zeros((3, 3), np.float32))


@pytest.mark.parametrize("group,with_prev", [(None, False), (4, True), (2, False)])
def test_weighted_svd_move_matches_transform(group, with_prev):
    """hreg_weighted_svd_tr (weighted_svd(move=)): R_, t_, R, t and the moved points are bitwise
    weighted_svd followed by transform, per batch group and with a previous transform composed."""
    from pcd_reg_hregnet_amd import engine
    rng = np.random.default_rng(9)
    B, n, n2 = 8, 256, 512
    src = dev(rng.uniform(-20, 20, (B, n, 3)).astype(np.float32))
    cor = dev(rng.uniform(-20, 20, (B, n, 3)).astype(np.float32))
    w = dev(rng.uniform(0.1, 1.0, (B, n)).astype(np.float32))
    pts = dev(rng.uniform(-20, 20, (B, n2, 3)).astype(np.float32))
    prev = None
    if with_prev:
        _, _, pR, pt = engine.weighted_svd(cor, src, w)
        prev = (pR, pt)
    a = engine.weighted_svd(src, cor, w, prev=prev, group=group)
    ref_moved = engine.transform(pts, a[2], a[3])
    b = engine.weighted_svd(src, cor, w, prev=prev, group=group, move=pts)
    torch.cuda.synchronize()
    for x, y in zip(a, b[:4]):
        assert torch.equal(x, y)
    assert torch.equal(ref_moved, b[4])


def test_transform_points():
    from pcd_reg_hregnet_amd import engine
    rng = np.random.default_rng(8)
    x = rng.normal(size=(2, 100, 3)).astype(np.float32)
    R = rng.normal(size=(2, 3, 3)).astype(np.float32)
    t = rng.normal(size=(2, 3)).astype(np.float32)
    out = engine.transform(dev(x), dev(R), dev(t)).cpu().numpy()
    np.testing.assert_allclose(out, np.einsum("bij,bnj->bni", R, x) + t[:, None], rtol=1e-5,
                               atol=1e-5)


@pytest.mark.parametrize("n", [16384, 5001, 600])
def test_spatial_index_morton_order(n):
    """hreg_spatial_index (clouds <= 16384 points): every point exactly once, in ascending
    18-bit Morton prefix order, ties by index (the stable radix passes), the block boxes
    enclosing their points."""
    from pcd_reg_hregnet_amd import _lib, engine, synthetic
    p = synthetic.lidar_batch(1, 16384, seed0=3)[1][:, :n]
    p = np.concatenate([p, np.random.default_rng(1).uniform(-40, 40, (1, n, 3)).astype(np.float32)], 0)
    nb = p.shape[0]
    ws = torch.empty(engine.spatial_index_bytes(nb, n), dtype=torch.uint8, device="cuda")
    _lib.call("hreg_spatial_index", torch.from_numpy(np.ascontiguousarray(p)).cuda(), nb, n, ws,
              _lib.stream_handle())
    torch.cuda.synchronize()
    np_ = 64
    while np_ < n:
        np_ *= 2
    raw = ws.cpu().numpy()
    spts = raw[:nb * np_ * 16].view(np.float32).reshape(nb, np_, 4)
    boxes = raw[nb * np_ * 16:].view(np.float32).reshape(nb, np_ // 64, 2, 4)
    for c in range(nb):
        ids = spts[c, :n, 3].view(np.int32)
        assert np.array_equal(np.sort(ids), np.arange(n))
        P = p[c]
        np.testing.assert_array_equal(spts[c, :n, :3], P[ids])
        lo, hi = P.min(0), P.max(0)
        sc = np.where(hi > lo, np.float32(1023.99) / (hi - lo), np.float32(0)).astype(np.float32)
        t = ((P - lo) * sc).astype(np.float32)
        qz = np.where(t <= 0, 0, np.where(t >= 1023, 1023, t.astype(np.int64)))
        code = np.zeros(n, np.int64)
        for b in range(10):
            for d in range(3):
                code |= ((qz[:, d] >> b) & 1) << (3 * b + d)
        key = (code[ids] >> 12) * n + ids
        assert np.all(np.diff(key) > 0)
        for b in range((n + 63) // 64):
            blk = spts[c, b * 64:min(n, b * 64 + 64), :3]
            assert np.all(boxes[c, b, 0, :3] <= blk.min(0)) and np.all(boxes[c, b, 1, :3] >= blk.max(0))


@pytest.mark.parametrize("case", ["lidar", "cube", "dups", "ragged", "lidar64k", "ragged64k"])
@pytest.mark.parametrize("K", [8, 32, 64])
def test_knn_group_indexed_matches_bruteforce(case, K):
    """The Morton-indexed, box-culled kNN grouping is bit-identical to the full scan
    (indices, relative coordinates, distances), ties included."""
    from pcd_reg_hregnet_amd import engine, synthetic
    rng = np.random.default_rng(7)
    if case == "lidar":
        p = synthetic.lidar_batch(2, 16384, seed0=3)[1]
    elif case == "cube":
        p = synthetic.cube_batch(2, 8192, seed=5)[0]
    elif case == "dups":  # heavy exact duplicates and a lattice: many equal distances
        base = rng.integers(-20, 20, (2, 1500, 3)).astype(np.float32)
        p = base[:, rng.integers(0, 1500, 6000)]
    elif case == "lidar64k":  # Model_V2's config 5 (n > 16384: the HBM-scatter index)
        p = synthetic.lidar_batch(1, 65536, seed0=4)[0]
    elif case == "ragged64k":
        p = rng.uniform(-40, 40, (2, 65536 - 37, 3)).astype(np.float32)
    else:  # n not a multiple of 64
        p = rng.uniform(-40, 40, (3, 5001, 3)).astype(np.float32)
    nb, n, _ = p.shape
    m = 300
    q = np.concatenate([p[:, rng.integers(0, n, m - 40)],
                        rng.uniform(-50, 50, (nb, 40, 3)).astype(np.float32)], 1)
    P = torch.from_numpy(np.ascontiguousarray(p)).cuda()
    Q = torch.from_numpy(np.ascontiguousarray(q)).cuda()
    ws = torch.empty(engine.spatial_index_bytes(nb, n), dtype=torch.uint8, device="cuda")
    a = engine.knn_group_indexed(Q, P, K, ws)
    b = engine.knn_group(Q, P, K)
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize("c", range(int(load_npz("transformation_loss.npz")["ncases"])))
def test_transformation_loss_matches_reference(c):
    """hreg_transformation_loss vs the reference losses.py:97-164 run (A16)."""
    from test_oracle_golden import LOSS, check_loss
    from pcd_reg_hregnet_amd import transformation_loss
    for i in range(LOSS[f"c{c}_pred_R"].shape[0]):
        args = [torch.from_numpy(LOSS[f"c{c}_{k}"][i]).cuda()
                for k in ("pred_R", "pred_t", "gt_R", "gt_t")]
        res = transformation_loss(*args, alpha=float(LOSS["alpha"]))
        check_loss([r.cpu().numpy() for r in res], c, i)


def test_transformation_loss_deterministic_and_checked():
    from pcd_reg_hregnet_amd import calc_rot_rre_err, calc_tran_rte_err, transformation_loss
    rng = np.random.default_rng(3)
    B = 1000
    pR = torch.from_numpy(rng.normal(size=(B, 3, 3)).astype(np.float32)).cuda()
    gR = torch.from_numpy(rng.normal(size=(B, 3, 3)).astype(np.float32)).cuda()
    pt = torch.from_numpy(rng.normal(size=(B, 3)).astype(np.float32)).cuda()
    gt = torch.from_numpy(rng.normal(size=(B, 3)).astype(np.float32)).cuda()
    # non-rotation inputs: asin of |E02| > 1 is NaN (as in the reference); NaN == NaN here
    a = [r.cpu().numpy() for r in transformation_loss(pR, pt, gR, gt)]
    b = [r.cpu().numpy() for r in transformation_loss(pR, pt, gR, gt)]
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    R_err, geo = calc_rot_rre_err(pR, gR)
    np.testing.assert_array_equal(R_err.cpu().numpy(), a[3])
    np.testing.assert_array_equal(geo.cpu().numpy(), a[4])
    T_err, eucl = calc_tran_rte_err(pt, gt)
    np.testing.assert_array_equal(T_err.cpu().numpy(), a[5])
    np.testing.assert_array_equal(eucl.cpu().numpy(), a[6])
    with pytest.raises(ValueError):
        transformation_loss(pR.cpu(), pt, gR, gt)
    with pytest.raises(ValueError):
        transformation_loss(pR[:, :2], pt, gR, gt)


def test_transformation_loss_differentiable_like_reference():
    """transformation_loss is differentiable in pred_R / pred_t, as the
    reference (losses.py:117-134): loss, loss_R and loss_t gradients against the
    reference formula in float64 torch autograd; values equal the forward-only call."""
    from pcd_reg_hregnet_amd import transformation_loss
    rng = np.random.default_rng(4)
    B, alpha = 6, 0.7
    R0 = torch.from_numpy(rng.normal(size=(B, 3, 3)).astype(np.float32))
    gR = torch.from_numpy(rng.normal(size=(B, 3, 3)).astype(np.float32)).cuda()
    t0 = torch.from_numpy(rng.normal(size=(B, 3)).astype(np.float32))
    gt = torch.from_numpy(rng.normal(size=(B, 3)).astype(np.float32)).cuda()
    plain = transformation_loss(R0.cuda(), t0.cuda(), gR, gt, alpha)
    for which in range(3):
        R = R0.cuda().requires_grad_(True)
        t = t0.cuda().requires_grad_(True)
        res = transformation_loss(R, t, gR, gt, alpha)
        torch.testing.assert_close(res[which].detach(), plain[which], rtol=1e-6, atol=1e-7)
        res[which].backward()
        R64 = R0.double().requires_grad_(True)
        t64 = t0.double().requires_grad_(True)
        eye = torch.eye(3, dtype=torch.float64).expand(B, 3, 3)
        lR = torch.norm(R64.transpose(2, 1) @ gR.cpu().double() - eye, dim=(1, 2)).mean()
        lt = torch.norm(t64 - gt.cpu().double(), dim=1).mean()
        (alpha * lR + lt, lR, lt)[which].backward()
        for ours, ref, x in ((R.grad, R64.grad, R64), (t.grad, t64.grad, t64)):
            got = torch.zeros_like(x) if ours is None else ours.cpu().double()
            want = torch.zeros_like(x) if ref is None else ref
            torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-6)


def test_fps_cluster_timeout_flags_and_leaves_valid_indices():
    """when the multi-workgroup FPS exchange times out (here forced: one
    participant never publishes, 2000 polls), the device status word reports it, the
    engine raises at its next check, and every idx entry is a valid index (0 fill)."""
    from pcd_reg_hregnet_amd import _lib as L, engine
    assert L.device_status(clear=True) == 0
    rng = np.random.default_rng(5)
    B, n, m = 2, 4096, 64
    x = dev(rng.uniform(-40, 40, (B, n, 3)).astype(np.float32))
    idx = torch.full((B, m), -7, dtype=torch.int32, device="cuda")
    smp = torch.empty((B, m, 3), device="cuda")
    temp = torch.empty((B, n), device="cuda")
    # no stall: the forced cluster kernel agrees with the oracle and raises nothing
    L.call("hreg_debug_fps_cluster", B, n, m, x, temp, idx, smp, -1, 1 << 22, L.stream_handle())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(idx.cpu().numpy(), oracle.fps(x.cpu().numpy(), m, None))
    assert L.device_status(clear=True) == 0
    idx.fill_(-7)
    # (participant 1: at n = 4096 the 32-slot cluster has 2 participants)
    L.call("hreg_debug_fps_cluster", B, n, m, x, temp, idx, smp, 1, 2000, L.stream_handle())
    torch.cuda.synchronize()
    got = idx.cpu().numpy()
    assert ((got >= 0) & (got < n)).all()
    assert (got[:, 1:] == 0).all()  # the exchange never completes: every later entry is 0
    assert np.isfinite(smp.cpu().numpy()).all()
    engine._status_pending = True
    with pytest.raises(RuntimeError, match="timed out"):
        engine.check_device_status()
    assert L.device_status(clear=True) == 0  # the check cleared it


def test_fps_cluster_timeout_seen_from_side_stream_without_sync():
    """the forced-stall cluster FPS launched on a non-blocking torch stream;
    engine.check_device_status() with no explicit synchronize still raises (the status
    read waits for the device), and the flag is consumed exactly once."""
    from pcd_reg_hregnet_amd import _lib as L, engine
    assert L.device_status(clear=True) == 0
    rng = np.random.default_rng(6)
    B, n, m = 2, 4096, 64
    x = dev(rng.uniform(-40, 40, (B, n, 3)).astype(np.float32))
    idx = torch.full((B, m), -7, dtype=torch.int32, device="cuda")
    smp = torch.empty((B, m, 3), device="cuda")
    temp = torch.empty((B, n), device="cuda")
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        L.call("hreg_debug_fps_cluster", B, n, m, x, temp, idx, smp, 1, 20000, L.stream_handle())
    engine._status_pending = True
    with pytest.raises(RuntimeError, match="timed out"):
        engine.check_device_status()
    got = idx.cpu().numpy()
    assert ((got >= 0) & (got < n)).all()
    assert L.device_status(clear=True) == 0


def test_engine_fps_weighted_mid_size():
    """weighted FPS for 8192 < n <= 16384 (no single-workgroup register case)
    through engine.fps / grouping(weights=...) matches the oracle."""
    from pcd_reg_hregnet_amd import engine
    rng = np.random.default_rng(9)
    B, m = 2, 256
    for n in (12000, 16384):
        xyz = rng.uniform(-40, 40, (B, n, 3)).astype(np.float32)
        w = rng.uniform(0.1, 2.0, (B, n)).astype(np.float32)
        idx, _ = engine.fps(dev(xyz), m, weights=dev(w))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(idx.cpu().numpy(), oracle.fps(xyz, m, w))
    engine.check_device_status()


@pytest.mark.parametrize("K", [8, 64])
def test_knn_points_ragged_lengths(K):
    """knn_points(lengths1, lengths2) (pytorch3d's ragged batches, r6): every cloud's valid
    rows are the dense kernel's selections over its first lengths2[b] points (oracle.knn on
    the sliced clouds, bit-exact); padded rows and slots beyond lengths2 are dist 0 / idx -1
    (padding values parity unpinned); return_nn / knn_gather(lengths) zero those slots."""
    from pcd_reg_hregnet_amd.knn import knn_gather, knn_points
    rng = np.random.default_rng(K)
    B, N1, N2 = 4, 300, 500
    p1 = rng.normal(size=(B, N1, 3)).astype(np.float32)
    p2 = rng.normal(size=(B, N2, 3)).astype(np.float32)
    l1 = np.array([300, 0, 17, 250])
    l2 = np.array([500, 40, 5, 64])
    d, i, nn = knn_points(dev(p1), dev(p2), lengths1=dev(l1), lengths2=dev(l2), K=K, return_nn=True)
    d, i, nn = d.cpu().numpy(), i.cpu().numpy(), nn.cpu().numpy()
    for b in range(B):
        if l1[b]:
            rd, ri = oracle.knn(p1[b:b + 1, :l1[b]], p2[b:b + 1, :l2[b]], K)
            np.testing.assert_array_equal(i[b, :l1[b]], ri[0])
            np.testing.assert_array_equal(d[b, :l1[b]], rd[0])
            want_nn = oracle.knn_gather(p2[b:b + 1, :l2[b]], np.maximum(ri, 0))[0]
            want_nn[ri[0] < 0] = 0.0  # slots beyond the cloud's points
            np.testing.assert_array_equal(nn[b, :l1[b]], want_nn)
        assert (i[b, l1[b]:] == -1).all() and (d[b, l1[b]:] == 0).all()
    # knn_gather's own lengths mask on a dense index
    idx = rng.integers(0, N2, (B, 7, K)).astype(np.int64)
    out = knn_gather(dev(p2), dev(idx), lengths=dev(l2)).cpu().numpy()
    want = oracle.knn_gather(p2, idx)
    want[np.broadcast_to(np.arange(K)[None, None, :] >= l2[:, None, None], want.shape[:3])] = 0.0
    np.testing.assert_array_equal(out, want)
