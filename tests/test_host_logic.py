"""Host-side logic of the HIP path, checked on the CPU: BN folding, the correspondence
heads' column permutations, the MFMA fragment tables of the fused level-1 kernel (by
emulating v_mfma_f32_32x32x2_f32 lane maps), weights, state-dict keys, synthetic data."""
import numpy as np
import pytest
import torch

from helpers import Args, state_dict_torch


@pytest.fixture(scope="module")
def P():
    from pcd_reg_hregnet_amd import engine
    from pcd_reg_hregnet_amd.models import HRegNet
    m = HRegNet(Args())
    m.load_state_dict(state_dict_torch())
    return m, engine.PreparedWeights(m.state_dict(), torch.device("cpu"))


def test_state_dict_keys_match_reference_checkpoint():
    """feature_extraction.* keys == ckpt/pretrained/nusc_feats.pth keys (192)."""
    from pcd_reg_hregnet_amd import weights
    from pcd_reg_hregnet_amd.models import HRegNet
    feats = weights.load_feats_npz()
    assert feats is not None and len(feats) == 192
    sd = HRegNet(Args()).state_dict()
    fe = {k[len("feature_extraction."):] for k in sd if k.startswith("feature_extraction.")}
    assert fe == set(feats)
    for k, v in feats.items():
        assert tuple(sd["feature_extraction." + k].shape) == tuple(v.shape), k
    n_params = sum(p.numel() for p in HRegNet(Args()).parameters())
    assert n_params == 2467846  # SURVEY.md 5 (DDP all-reduce size)


def test_model_v2_state_dict_layout():
    """Model_V2 = HRegNet's parameters + fine_corres_2.mlpx (model_v2/layers.py:460-462:
    Conv1d(256->128, bias) + BatchNorm1d(128)); the V2 fixture weights load strictly."""
    from helpers import state_dict_v2_torch
    from pcd_reg_hregnet_amd.models import HRegNet, Model_V2
    v2 = Model_V2(Args())
    extra = set(v2.state_dict()) - set(HRegNet(Args()).state_dict())
    assert extra == {"fine_corres_2.mlpx.0.weight", "fine_corres_2.mlpx.0.bias",
                     "fine_corres_2.mlpx.1.weight", "fine_corres_2.mlpx.1.bias",
                     "fine_corres_2.mlpx.1.running_mean", "fine_corres_2.mlpx.1.running_var",
                     "fine_corres_2.mlpx.1.num_batches_tracked"}
    assert tuple(v2.state_dict()["fine_corres_2.mlpx.0.weight"].shape) == (128, 256, 1)
    assert sum(p.numel() for p in v2.parameters()) == 2467846 + 256 * 128 + 128 + 2 * 128
    v2.load_state_dict(state_dict_v2_torch())


def test_weights_deterministic():
    a = state_dict_torch()
    b = state_dict_torch()
    assert all(torch.equal(a[k], b[k]) for k in a)


def test_bn_fold_matches_torch_eval(P):
    m, prep = P
    bn = m.feature_extraction.detector_2.convs[1].eval()
    conv = m.feature_extraction.detector_2.convs[0]
    x = torch.randn(2, 68, 16, 8)
    ref = bn(conv(x))
    lin = prep.det[1][0]
    acc = torch.einsum("oc,bcmk->bomk", lin.W, x)
    got = acc * lin.alpha.view(1, -1, 1, 1) + lin.beta.view(1, -1, 1, 1)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("C,kind", [(256, "coarse"), (128, "fine"), (64, "fine")])
def test_head_column_permutations(C, kind):
    """W[:, perm] applied to the packed small-feature layout == W applied to the
    reference concat order (layers.py:364-380, 444-445)."""
    from pcd_reg_hregnet_amd import engine
    rng = np.random.default_rng(C)
    K = 2 * C + (16 if kind == "coarse" else 12)
    W = rng.normal(size=(8, K))
    feats_ref = rng.normal(size=(5, K))
    if kind == "coarse":
        perm = engine._perm_coarse(C)
    else:
        perm = engine._perm_fine(C)
    assert sorted(perm) == list(range(K))
    packed = feats_ref[:, perm]
    np.testing.assert_allclose(packed @ W[:, perm].T, feats_ref @ W.T, rtol=1e-12)
    # the packed layout the kernels produce: [geom10, w_src, w_dst, (sims4), desc, knn_desc]
    if kind == "coarse":
        assert perm[10:16] == [10 + 2 * C, 11 + 2 * C, 12 + 2 * C, 13 + 2 * C, 14 + 2 * C,
                               15 + 2 * C]
    else:
        assert perm[10:12] == [10 + 2 * C, 11 + 2 * C]


def _mfma_32x32x2(a_lane, b_lane, acc):
    """Exact lane semantics of v_mfma_f32_32x32x2_f32 (cdna_hip_programming.md 3):
    A[i][k] = a[i + 32k], B[k][j] = b[j + 32k], D[i][j] += sum_k A[i][k] B[k][j];
    acc[l][q] <-> D[(q&3) + 8(q>>2) + 4(l>>5)][l&31]."""
    A = np.stack([a_lane[:32], a_lane[32:]], 1)          # [32 i][2 k]
    B = np.stack([b_lane[:32], b_lane[32:]], 0)          # [2 k][32 j]
    D = A @ B
    out = acc.copy()
    for l in range(64):
        for q in range(16):
            out[l, q] += D[(q & 3) + 8 * (q >> 2) + 4 * (l >> 5), l & 31]
    return out


def _to_acc(X):
    """[C=32*T][32 rows] activations -> accumulator layout [T][64 lanes][16]."""
    T = X.shape[0] // 32
    acc = np.zeros((T, 64, 16))
    for t in range(T):
        for l in range(64):
            for q in range(16):
                acc[t, l, q] = X[t * 32 + (q & 3) + 8 * (q >> 2) + 4 * (l >> 5), l & 31]
    return acc


def test_l1_fragment_tables_emulated():
    """frag_layer / frag_geom reproduce W @ X through the accumulator-chaining order of
    group_l1.hip (B operand of k-step q = the previous layer's accumulator register q)."""
    from pcd_reg_hregnet_amd import engine
    rng = np.random.default_rng(0)
    # a 64 -> 64 layer (2 input tiles, 2 output tiles) on 32 rows
    W = rng.normal(size=(64, 64)).astype(np.float32)
    X = rng.normal(size=(64, 32)).astype(np.float32)
    frag = engine.frag_layer(torch.from_numpy(W)).numpy().reshape(2, 2, 16, 64)
    xin = _to_acc(X.astype(np.float64))
    out = np.zeros((2, 64, 16))
    for co in range(2):
        for ct in range(2):
            for q in range(16):
                out[co] = _mfma_32x32x2(frag[co, ct, q].astype(np.float64), xin[ct][:, q], out[co])
    np.testing.assert_allclose(out, _to_acc(W.astype(np.float64) @ X), rtol=1e-10, atol=1e-9)
    # the first layer (4 geometric channels): k-step s, lane half h -> channel 2h + s
    W1 = rng.normal(size=(32, 4)).astype(np.float32)
    G = rng.normal(size=(32, 4)).astype(np.float32)   # [rows][4]
    f1 = engine.frag_geom(torch.from_numpy(W1)).numpy().reshape(2, 64)
    acc = np.zeros((64, 16))
    for s in range(2):
        b = np.array([G[l & 31, 2 * (l >> 5) + s] for l in range(64)], np.float64)
        acc = _mfma_32x32x2(f1[s].astype(np.float64), b, acc)
    np.testing.assert_allclose(acc, _to_acc((W1 @ G.T).astype(np.float64))[0], rtol=1e-6,
                               atol=1e-6)


def test_l1_table_size_matches_kernel(P):
    _, prep = P
    from pcd_reg_hregnet_amd import _lib
    L = _lib.load_checkers(require_gpu=False)  # (test-only checker library)
    assert prep.l1_table.numel() == L.hreg_group_l1_table_floats()


def test_synthetic_pairs_deterministic_and_shaped():
    from pcd_reg_hregnet_amd import synthetic
    a = synthetic.lidar_batch(2, 4096, seed0=5)
    b = synthetic.lidar_batch(2, 4096, seed0=5)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    s, d, R, t = a
    assert s.shape == (2, 4096, 3) and d.shape == (2, 4096, 3) and s.dtype == np.float32
    np.testing.assert_allclose(R[0] @ R[0].T, np.eye(3), atol=1e-5)
    assert np.linalg.norm(d, axis=-1).max() <= 80.5
    # ~2 % exact duplicates exercise FPS/kNN ties
    u = np.unique(d[0], axis=0).shape[0]
    assert 0.95 * 4096 < u < 4096
    # the generator's perturbation is the dataset's: |angle| <= 20 deg, |t| <= 0.5 m per axis
    ang = np.degrees(np.arccos(np.clip((np.trace(R, axis1=1, axis2=2) - 1) / 2, -1, 1)))
    assert np.all(ang <= 20 * np.sqrt(3) + 1e-3) and np.all(np.abs(t) <= 0.5)


def test_l2_input_fragments_emulated():
    """frag_input: the first level-2 layer over [geom 4 | feature CF] as group_l2.hip feeds
    it (geom k-step s, half h -> channel 2h+s; feature k-step s, half h -> 4 + h*CF/2 + s)."""
    from pcd_reg_hregnet_amd import engine
    rng = np.random.default_rng(1)
    CF, Cout = 64, 64
    W = rng.normal(size=(Cout, 4 + CF)).astype(np.float32)
    X = rng.normal(size=(32, 4 + CF)).astype(np.float32)     # [rows][channels]
    fg, ff = (t.numpy() for t in engine.frag_input(torch.from_numpy(W)))
    T1, TF = Cout // 32, CF // 2
    fg = fg.reshape(T1, 2, 64)
    ff = ff.reshape(T1, TF, 64)
    acc = np.zeros((T1, 64, 16))
    for co in range(T1):
        for s in range(2):
            b = np.array([X[l & 31, 2 * (l >> 5) + s] for l in range(64)], np.float64)
            acc[co] = _mfma_32x32x2(fg[co, s].astype(np.float64), b, acc[co])
        for s in range(TF):
            b = np.array([X[l & 31, 4 + (l >> 5) * TF + s] for l in range(64)], np.float64)
            acc[co] = _mfma_32x32x2(ff[co, s].astype(np.float64), b, acc[co])
    np.testing.assert_allclose(acc, _to_acc((W.astype(np.float64) @ X.T.astype(np.float64))),
                               rtol=1e-9, atol=1e-9)


def test_l2_table_size_matches_kernel(P):
    _, prep = P
    from pcd_reg_hregnet_amd import _lib
    L = _lib.load_checkers(require_gpu=False)  # (test-only checker library)
    assert prep.l2_table.numel() == L.hreg_group_l2_table_floats()


def test_l3_table_size_matches_kernel(P):
    _, prep = P
    from pcd_reg_hregnet_amd import _lib
    L = _lib.load_checkers(require_gpu=False)  # (test-only checker library)
    assert prep.l3_table.numel() == L.hreg_group_l3_table_floats()


def test_split_tables_match_kernel(P):
    """group_split.hip tables: the chained kernel's fragments regrouped 4 k-steps per lane
    (2 for the geometry block), plus mlp1's x2 block row-major [CM1][C3] (the per-group
    matrix-vector product) before the epilogues."""
    _, prep = P
    from pcd_reg_hregnet_amd import _lib
    L = _lib.load_checkers(require_gpu=False)  # (test-only checker library)
    assert prep.l2s_table.numel() == L.hreg_group_split_l2_table_floats()
    assert prep.l3s_table.numel() == L.hreg_group_split_l3_table_floats()
    for a, b, lvl in ((prep.l2_table, prep.l2s_table, 1), (prep.l3_table, prep.l3s_table, 2)):
        a, b = a.cpu(), b.cpu()
        x2 = prep.desc_mlp[lvl][0].W[:, :prep.det[lvl][2].N].reshape(-1).cpu()
        ne = sum(2 * lin.N for lin in (*prep.det[lvl], *prep.desc[lvl], *prep.desc_mlp[lvl]))
        nf = b.numel() - x2.numel() - ne  # b = [fragments][x2 block][epilogues]
        assert torch.equal(b[nf:nf + x2.numel()], x2)
        bx = torch.cat([b[:nf], b[nf + x2.numel():]])
        assert bx.numel() == a.numel()
        assert torch.equal(torch.sort(a).values, torch.sort(bx).values)


def test_fine_head_table_sizes_match_kernel(P):
    _, prep = P
    from pcd_reg_hregnet_amd import _lib
    L = _lib.load(require_gpu=False)
    assert prep.fine_table["fine_corres_1"].numel() == L.hreg_fine_head_table_floats(64)
    assert prep.fine_table["fine_corres_2"].numel() == L.hreg_fine_head_table_floats(128)


def test_nbr_head_table_size_matches_kernel(P):
    _, prep = P
    from pcd_reg_hregnet_amd import _lib
    L = _lib.load(require_gpu=False)
    assert prep.nbr_table.numel() == L.hreg_nbr_head_table_floats()


def test_split_tables6_match_kernel(P):
    _, prep = P
    from pcd_reg_hregnet_amd import _lib
    L = _lib.load(require_gpu=False)
    assert prep.l2s_table6.numel() == L.hreg_group_split6_l2_table_floats()
    assert prep.l3s_table6.numel() == L.hreg_group_split6_l3_table_floats()


def test_mlp_head_tables6_match_kernel(P):
    _, prep = P
    from pcd_reg_hregnet_amd import _lib
    L = _lib.load(require_gpu=False)
    sizes = {C: L.hreg_mlp_head6_table_floats(C) for C in (64, 128, 256, 512)}
    assert sorted(t.numel() for t in prep.head_table6.values()) == sorted(
        [sizes[64], sizes[128], sizes[256], sizes[512], sizes[256], sizes[128]])


def test_coarse_table6_matches_kernel(P):
    _, prep = P
    from pcd_reg_hregnet_amd import _lib
    L = _lib.load(require_gpu=False)
    assert prep.coarse_table6.numel() == L.hreg_coarse_head6_table_floats()


def test_l1_table6_matches_kernel(P):
    _, prep = P
    from pcd_reg_hregnet_amd import _lib
    L = _lib.load(require_gpu=False)
    assert prep.l1_table6.numel() == L.hreg_group_l1_6_table_floats()


def test_head6_tables_match_kernel(P):
    """bf16x6 head tables (engine.fine_head_table6 / nbr_head_table6): sizes match the
    kernels' Head6Cfg, and the three bf16 pieces of every weight sum back to it exactly."""
    _, prep = P
    from pcd_reg_hregnet_amd import _lib, engine
    L = _lib.load(require_gpu=False)
    assert prep.fine_table6["fine_corres_1"].numel() == L.hreg_head6_table_floats(128)
    assert prep.fine_table6["fine_corres_2"].numel() == L.hreg_head6_table_floats(256)
    # the channel-split correspondence kernel reads the same tables (hreg_corr_head6)
    assert prep.fine_table6["fine_corres_1"].numel() == L.hreg_corr_head6_table_floats(128)
    assert prep.fine_table6["fine_corres_2"].numel() == L.hreg_corr_head6_table_floats(256)
    assert prep.coarse_table6.numel() == L.hreg_corr_head6_table_floats(512)
    assert L.hreg_corr_head6_table_floats(64) == -1
    assert prep.nbr_table6.numel() == L.hreg_head6_table_floats(256)
    W = prep.coarse_convs2[1].W.cpu()
    pieces = engine._bf16_pieces(W).to(torch.int32) << 16
    back = [p.view(torch.float32).double() for p in pieces]
    assert torch.equal(back[0] + back[1] + back[2], W.double())


def test_level1_prefetch_key_identity_and_version():
    """a level-1 prefetch must not be reused when the same buffers hold new
    data (copy_ into a static input) or when a new tensor reuses a freed address."""
    from pcd_reg_hregnet_amd.trainer import Level1Prefetch
    pf = Level1Prefetch.__new__(Level1Prefetch)
    pf.key = pf.prepared = None
    s, d = torch.zeros(2, 8, 3), torch.zeros(2, 8, 3)
    pf.key = Level1Prefetch._key(s, d)
    assert pf.matches(s, d)
    assert not pf.matches(d, s)
    assert not pf.matches(s.clone(), d)          # another object, same contents
    assert not pf.matches(s.view(2, 8, 3), d)    # an alias is another object too
    s.copy_(torch.ones_like(s))                  # static buffer refilled in place
    assert not pf.matches(s, d)
    pf.key = Level1Prefetch._key(s, d)
    d[0, 0, 0] = 5.0
    assert not pf.matches(s, d)
    # a dead tensor never matches, whatever lives at its address now
    a, b = torch.zeros(4, 8, 3), torch.zeros(4, 8, 3)
    pf.key = Level1Prefetch._key(a, b)
    del a
    assert pf.key[0]() is None
    pf.discard()
    assert pf.key is None and not pf.matches(s, d)


def test_bench_times_every_mfma_entry_the_engine_calls():
    """bench.MfmaTimer brackets the level / head kernels by C-ABI entry name: every fused
    level or head entry engine.py can launch must be in bench.MFMA_ENTRIES, or the roofline
    family silently drops it (r3: hreg_group_split6j_l3 / hreg_corr_head6x / hreg_nbr_head6sx
    were missing, so the level-3 launches fell out of `roofline.achieved`)."""
    import os
    import re
    import bench
    src = open(os.path.join(os.path.dirname(os.path.dirname(__file__)), "pcd_reg_hregnet_amd",
                            "engine.py")).read()
    names = set(re.findall(r'"(hreg_(?:group_l\d\w*|group\d?\w*_l\d|group_split\w*|\w*head\d?\w*))"', src))
    names -= {"hreg_head_out"}
    names = {n for n in names if not n.endswith("_table_floats")}
    assert "hreg_group_split6j_l3" in names and "hreg_corr_head6x" in names
    missing = sorted(n for n in names if n not in bench.MFMA_ENTRIES)
    assert not missing, missing


def test_bench_entry_peaks():
    """Every timed MFMA entry is priced at its kernel's peak: the bf16x6 kernels (built on
    mfma_chain.h / split_chain.h, v_mfma_f32_32x32x16_bf16) at the bf16 dense peak / 6, the
    fp32-MFMA kernels at the f32 matrix peak.  r3: hreg_group_split6j_l3, hreg_corr_head6x and
    hreg_nbr_head6sx were priced at the fp32 peak (roofline.frac 0.71 instead of 0.45)."""
    import bench
    b6 = {"hreg_group_l1_6", "hreg_group_l1_6g", "hreg_group6_l2",
          "hreg_group_split6_l2", "hreg_group_split6_l3", "hreg_group_split6j_l3",
          "hreg_group6_l3",
          "hreg_fine_head6", "hreg_nbr_head6", "hreg_nbr_head6s", "hreg_nbr_head6sx",
          "hreg_coarse_head6", "hreg_corr_head6", "hreg_corr_head6x", "hreg_mlp_head6", "hreg_mlp_head6x",
              "hreg_gemm6"}
    for name in set(bench.MFMA_ENTRIES) | {"hreg_gemm", "hreg_gemm6"}:
        want = bench.PEAK_B6_TFLOPS if name in b6 else bench.PEAK_FP32_MFMA_TFLOPS
        assert bench.entry_peak(name) == want, name


def test_graph_executor_refuses_too_few_hw_queues():
    """the graph executor refuses GPU_MAX_HW_QUEUES below 4 (2 crashed the
    HIP runtime in r4's 20-lane replay) with a clear error before any capture; unset, invalid
    and the measured 4 / 8 / 16 pass; a single-stream executor is not affected."""
    import pytest
    from pcd_reg_hregnet_amd import engine
    w = engine.fork_width(20, True, True)
    assert w == 41
    assert engine.fork_width(4, False, False) == 8
    for env in ({}, {"GPU_MAX_HW_QUEUES": "4"}, {"GPU_MAX_HW_QUEUES": "16"},
                {"GPU_MAX_HW_QUEUES": "x"}):
        assert engine.check_hw_queues(w, env) >= 4
    for q in ("1", "2", "3"):
        with pytest.raises(RuntimeError, match="GPU_MAX_HW_QUEUES"):
            engine.check_hw_queues(w, {"GPU_MAX_HW_QUEUES": q})
    assert engine.check_hw_queues(1, {"GPU_MAX_HW_QUEUES": "2"}) == 2


def test_bench_default_merge_divides_steps():
    """bench.default_merge: the largest divisor of --steps up to the model's merge factor, so
    the timed region is always exactly --steps reference batches (the driver's 20, the default
    48, and step counts the factor does not divide)."""
    import bench
    assert bench.HREGNET_MERGE == 4 and bench.V2_MERGE == 12
    for steps, want in ((20, 4), (48, 4), (10, 2), (7, 1), (9, 3), (1, 1)):
        assert bench.default_merge(steps, False) == want, steps
    for steps, want in ((48, 12), (20, 10), (16, 8), (7, 7), (13, 1)):
        assert bench.default_merge(steps, True) == want, steps
    for steps in range(1, 100):
        for v2 in (False, True):
            m = bench.default_merge(steps, v2)
            assert steps % m == 0 and 1 <= m <= (12 if v2 else 4)


def _fake_forward_inputs(bench, v2):
    import argparse
    args = argparse.Namespace(steps=20, warmup=8, executor="graph", lanes=5, points=65536 if v2 else 16384,
                              model="v2" if v2 else "hregnet", batch=2 if v2 else 8)
    # MfmaTimer.result per kind: (ms, launches, FLOPs, bytes, executed FLOPs)
    res = {k: (10.0 + i, 40 + i, 3e12 + i, 1e9, 2.5e12) for i, k in enumerate(bench.MfmaTimer.KINDS)}
    ent = {name: {"launches_per_step": 1.0, "avg_launch_us": 500.0, "tflops": 200.0,
                  "peak": bench.entry_peak(name), "_ms": 10.0, "_flops": 2e12}
           for name in ("hreg_group_l1_6", "hreg_group6_l2", "hreg_group_split6j_l3", "hreg_mlp_head6x")}
    return args, res, ent


def _check_line(line, metric_word):
    import json
    d = json.loads(json.dumps(line))  # serialisable, nothing left as a tensor / numpy scalar
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert metric_word in d["metric"] and d["unit"] == "pairs/s" and d["higher_is_better"] is True
    assert "workload" in d["config"]
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    return d


@pytest.mark.parametrize("model", ["hregnet", "v2", "b32"])
def test_bench_forward_line_assembles_on_cpu(model):
    """every bench mode's JSON line is assembled by a pure function from its
    measurements, so a NameError in the assembly (r5's bench_train `merge`) fails here, on the
    CPU, before it can reach a GPU run.  b32: configs[2] (bench.py --batch 32)."""
    import bench
    v2 = model == "v2"
    args, res, ent = _fake_forward_inputs(bench, v2)
    if model == "b32":
        args.batch = 32
    line = bench.forward_line(
        args, v2=v2, B=args.batch, merge=4, world=1, value=8000.0, ms_per_step=1.0, host_submit_s=0.002,
        res=res, ent=ent, level_names=["a (level 1)", "b (level 2)", "c (level 3)"], traffic=(3e8, "x.json"),
        inexec=None, fps={"level1": {"us_per_iteration": 1.0}}, lat={"graph_ms": 2.7},
        cpu={"value": 1.8, "unit": "pairs/s", "cores": 16, "kind": "port", "sample": "s"}, bs1=True, fs=not v2,
        merge1=None if v2 else {"value": 7400.0, "ms_per_step": 1.08})
    d = _check_line(line, "Model_V2" if v2 else "HRegNet")
    assert d["value"] == 8000.0 and d["config"]["merge"] == 4
    assert ("configs[4]" if v2 else "configs[2]" if model == "b32" else "configs[1]") in d["config"]["workload"]
    assert d["cpu_baseline"]["kind"] == "port"


def test_bench_train_line_assembles_on_cpu():
    import argparse
    import bench
    args = argparse.Namespace(steps=10, warmup=2, points=16384, batch=8)
    line = bench.train_line(args, B=8, world=1, value=418.0, elapsed=0.19, losses=[1.44, 5.93],
                            nt=(80.0, 1000, 1e13), tn=(60.0, 900, 8e12), graphed=True)
    d = _check_line(line, "training")
    assert d["loss_first_last"] == [1.44, 5.93] and "configs[3]" in d["config"]["workload"]


@pytest.mark.parametrize("use_sim,use_neighbor", [(True, True), (True, False), (False, True), (False, False)])
def test_coarse_reg_variants_layout_and_padding(use_sim, use_neighbor):
    """CoarseReg(use_sim, use_neighbor) (layers.py:237-244): convs_1 over 2C + 16 / 14 / 14 / 12
    inputs, convs_2 present in every variant; PreparedWeights widens convs_1[0] to the 2C + 16
    layout with zero columns exactly where the variant has no similarity feature."""
    from pcd_reg_hregnet_amd import engine, models
    C = 256
    m = models.CoarseReg(8, C, use_sim, use_neighbor)
    W = m.convs_1[0].weight.detach().clone()
    assert W.shape[1] == 2 * C + 12 + 2 * use_sim + 2 * use_neighbor
    assert m.convs_2[0].weight.shape[1] == C + 4
    sd = {"coarse_corres.convs_1.0.weight": W.clone(), "coarse_corres.convs_2.0.weight": m.convs_2[0].weight}
    engine._pad_coarse_convs1(sd, use_sim, use_neighbor)
    W16 = sd["coarse_corres.convs_1.0.weight"]
    assert W16.shape[1] == 2 * C + 16
    assert torch.equal(W16[:, :2 * C + 12], W[:, :2 * C + 12])
    sims = W16[:, 2 * C + 12:]
    present = [use_sim, use_sim, use_neighbor, use_neighbor]
    src = iter(range(2 * C + 12, W.shape[1]))
    for j, p in enumerate(present):
        if p:
            assert torch.equal(sims[:, j], W[:, next(src)])
        else:
            assert not sims[:, j].any()
    with pytest.raises(ValueError):
        engine._pad_coarse_convs1({"coarse_corres.convs_1.0.weight": W[:, :-2].clone(),
                                   "coarse_corres.convs_2.0.weight": m.convs_2[0].weight}, use_sim, use_neighbor)
