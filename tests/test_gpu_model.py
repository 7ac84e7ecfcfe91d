"""End-to-end HRegNet forward on the GPU against the reference fixtures and the oracle.

Contract (BASELINE.json north_star; tests/parity.py): FPS level-1
indices bit-exact; every other FPS / kNN selection the reference's unless it is a
float64 near tie (relative margin <= 2e-5 WFPS / 1e-5 kNN) or downstream of one;
continuous outputs on the rows with identical selections within max(1e-5, 4 x the fp32
reference's own distance from its float64 replay); R/t within 1e-4 absolute.
"""
import numpy as np
import math

import pytest
import torch

from helpers import Args, load_npz, state_dict_torch
from test_oracle_golden import compare_forward

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def net():
    from pcd_reg_hregnet_amd.models import HRegNet
    m = HRegNet(Args())
    m.load_state_dict(state_dict_torch())
    return m.cuda().eval()


def _run(net, src, dst, record=False):
    """eager engine.hregnet_forward -> numpy dict; record: every kNN selection under "_knn"
    (engine.INDEX_RECORD)"""
    from pcd_reg_hregnet_amd import engine
    P = net.prepared(torch.device("cuda"))
    engine.INDEX_RECORD = {} if record else None
    try:
        with torch.no_grad():
            r = engine.hregnet_forward(P, torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda())
        torch.cuda.synchronize()
        if record:
            r["_knn"] = engine.INDEX_RECORD
    finally:
        engine.INDEX_RECORD = None

    def cpu(x):
        if isinstance(x, torch.Tensor):
            return x.cpu().numpy()
        if isinstance(x, list):
            return [cpu(v) for v in x]
        if isinstance(x, dict):
            return {k: cpu(v) for k, v in x.items()}
        return x
    return cpu(r)


@pytest.mark.parametrize("fixture", ["hregnet_lidar_b2_n4096.npz", "hregnet_cube_b1_n16384.npz"])
def test_forward_matches_reference_fixture(net, fixture):
    g = load_npz(fixture)
    r = _run(net, g["src"], g["dst"], record=True)
    B = g["src"].shape[0]
    np.testing.assert_array_equal(r["_fps_idx"][0][:B], g["src_fps_1"])
    np.testing.assert_array_equal(r["_fps_idx"][0][B:], g["dst_fps_1"])
    compare_forward(r, g, title="GPU vs " + fixture)


def test_random_sampling_forward_matches_reference(net):
    """use_fps=False (layers.py:144-147; the default of the reference's training scripts):
    the samples are torch.randperm draws on the host generator in the reference's order,
    so after the fixture's seed engine.hregnet_forward(use_fps=False) selects the
    reference's points and matches its forward under the parity contract; the module API
    (HRegNet with args.use_fps False) draws the same and returns the same bits."""
    from pcd_reg_hregnet_amd import engine
    from pcd_reg_hregnet_amd.models import HRegNet
    g = load_npz("hregnet_randsample_b2_n4096.npz")
    B = g["src"].shape[0]
    P = net.prepared(torch.device("cuda"))
    src, dst = torch.from_numpy(g["src"]).cuda(), torch.from_numpy(g["dst"]).cuda()
    torch.manual_seed(int(g["perm_seed"]))
    engine.INDEX_RECORD = {}
    try:
        with torch.no_grad():
            r = engine.hregnet_forward(P, src, dst, use_fps=False)
        torch.cuda.synchronize()
        rec = engine.INDEX_RECORD
    finally:
        engine.INDEX_RECORD = None
    cpu = {"rotation": [x.cpu().numpy() for x in r["rotation"]],
           "translation": [x.cpu().numpy() for x in r["translation"]],
           "_fps_idx": [x.cpu().numpy() for x in r["_fps_idx"]],
           "_knn": {k: v.cpu().numpy() for k, v in rec.items()}}
    for k in r:
        if k.startswith(("src_xyz_corres", "src_dst_weights")):
            cpu[k] = r[k].cpu().numpy()
    for part in ("src_feats", "dst_feats"):
        cpu[part] = {k: v.cpu().numpy() for k, v in r[part].items()}
    for lv in (1, 2, 3):
        np.testing.assert_array_equal(cpu["_fps_idx"][lv - 1][:B], g[f"src_fps_{lv}"])
        np.testing.assert_array_equal(cpu["_fps_idx"][lv - 1][B:], g[f"dst_fps_{lv}"])
    compare_forward(cpu, g, title="GPU vs hregnet_randsample_b2_n4096.npz")

    class NoFps(Args):
        use_fps = False
    m = HRegNet(NoFps())
    m.load_state_dict(net.state_dict())
    m = m.cuda().eval()
    torch.manual_seed(int(g["perm_seed"]))
    with torch.no_grad():
        r2 = m(src, dst)
    assert torch.equal(r2["rotation"][-1], r["rotation"][-1])


def test_module_forward_api(net):
    """HRegNet.forward returns the reference's dict and shapes (models.py:129-148)."""
    g = load_npz("hregnet_lidar_b2_n4096.npz")
    with torch.no_grad():
        r = net(torch.from_numpy(g["src"]).cuda(), torch.from_numpy(g["dst"]).cuda())
    B = 2
    assert [tuple(x.shape) for x in r["rotation"]] == [(B, 3, 3)] * 3
    assert [tuple(x.shape) for x in r["translation"]] == [(B, 3)] * 3
    for lv, n in ((3, 256), (2, 512), (1, 1024)):
        assert tuple(r[f"src_xyz_corres_{lv}"].shape) == (B, n, 3)
        assert tuple(r[f"src_dst_weights_{lv}"].shape) == (B, n)
    for part in ("src_feats", "dst_feats"):
        f = r[part]
        for lv, (m, c) in enumerate(((1024, 64), (512, 128), (256, 256)), 1):
            assert tuple(f[f"xyz_{lv}"].shape) == (B, m, 3)
            assert tuple(f[f"sigmas_{lv}"].shape) == (B, m)
            assert tuple(f[f"desc_{lv}"].shape) == (B, c, m)
    np.testing.assert_allclose(r["rotation"][-1].cpu().numpy(), g["R1"], atol=1e-4)


def test_batch_independence(net):
    """Pairs are independent in eval mode: a pair's output does not depend on the
    rest of the batch (the property multi-GPU sharding relies on)."""
    from pcd_reg_hregnet_amd import synthetic
    s, d, _, _ = synthetic.lidar_batch(3, 4096, seed0=10)
    full = _run(net, s, d)
    one = _run(net, s[1:2], d[1:2])
    for i in range(3):
        np.testing.assert_array_equal(full["rotation"][i][1], one["rotation"][i][0])
        np.testing.assert_array_equal(full["translation"][i][1], one["translation"][i][0])


def test_deterministic(net):
    from pcd_reg_hregnet_amd import synthetic
    s, d, _, _ = synthetic.lidar_batch(2, 4096, seed0=20)
    a = _run(net, s, d)
    b = _run(net, s, d)
    for i in range(3):
        np.testing.assert_array_equal(a["rotation"][i], b["rotation"][i])
        np.testing.assert_array_equal(a["translation"][i], b["translation"][i])


def _oracle_as_fixture(o, s, d):
    """the oracle's forward (with its kNN selections) in the fixture layout"""
    import parity
    g = parity.as_layout(o, s.shape[0])
    g["src"], g["dst"] = s, d
    return g


@pytest.mark.parametrize("B,seed0", [(8, 100), (32, 200)])
def test_vs_oracle_lidar(net, B, seed0):
    """BASELINE configs[1] (B=8) and configs[2] (B=32): KITTI-shape LiDAR pairs of 2 x 16384
    points, the whole batch through one forward, against the CPU oracle pair by pair."""
    from oracle import oracle
    from pcd_reg_hregnet_amd import synthetic
    from helpers import state_dict_numpy
    s, d, _, _ = synthetic.lidar_batch(B, 16384, seed0=seed0)
    r = _run(net, s, d, record=True)
    o = oracle.hregnet_forward(state_dict_numpy(), s, d)
    g = _oracle_as_fixture(o, s, d)
    np.testing.assert_array_equal(r["_fps_idx"][0][:B], o["src_feats"]["fps_idx_1"])
    np.testing.assert_array_equal(r["_fps_idx"][0][B:], o["dst_feats"]["fps_idx_1"])
    compare_forward(r, g, title=f"GPU vs oracle, B={B} N=16384")


def test_pipeline_matches_serial(net):
    """The pipelined executor runs level 1 on a side stream; outputs must be bitwise
    identical to the serial forward for every batch."""
    from pcd_reg_hregnet_amd import engine, synthetic
    P = net.prepared(torch.device("cuda"))
    batches = []
    for sd in (30, 31, 32):
        s, d, _, _ = synthetic.lidar_batch(2, 4096, seed0=sd)
        batches.append((torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()))
    with torch.no_grad():
        piped = engine.Pipeline(P, torch.device("cuda")).run(batches)
        serial = [engine.hregnet_forward(P, s, d) for s, d in batches]
    torch.cuda.synchronize()
    for a, b in zip(piped, serial):
        for i in range(3):
            assert torch.equal(a["rotation"][i], b["rotation"][i])
            assert torch.equal(a["translation"][i], b["translation"][i])
        assert torch.equal(a["src_feats"]["desc_1"], b["src_feats"]["desc_1"])


def test_graph_pipeline_matches_eager(net):
    """HIP-graph replay of the pipelined forward == the eager forward, bitwise."""
    from pcd_reg_hregnet_amd import engine, synthetic
    P = net.prepared(torch.device("cuda"))
    s, d, _, _ = synthetic.lidar_batch(2, 4096, seed0=40)
    src, dst = torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()
    with torch.no_grad():
        gp = engine.GraphPipeline(P, src, dst)
        ref = engine.hregnet_forward(P, src, dst)
        for steps in (1, 2, 5):
            out = gp.run(steps)
            torch.cuda.synchronize()
            for i in range(3):
                assert torch.equal(out["rotation"][i], ref["rotation"][i])
                assert torch.equal(out["translation"][i], ref["translation"][i])
        s2, d2, _, _ = synthetic.lidar_batch(2, 4096, seed0=41)
        gp.load(torch.from_numpy(s2).cuda(), torch.from_numpy(d2).cuda())
        out = gp.run(3)
        ref2 = engine.hregnet_forward(P, torch.from_numpy(s2).cuda(), torch.from_numpy(d2).cuda())
        torch.cuda.synchronize()
        assert torch.equal(out["rotation"][-1], ref2["rotation"][-1])


def test_chain_fork_matches_serial(net):
    """engine.chain_fork (the level-1 spatial index beside the FPS, the level-2/3 input
    projections beside their WFPS + kNN, each on a side stream): bitwise the serial forward."""
    from pcd_reg_hregnet_amd import engine, synthetic
    P = net.prepared(torch.device("cuda"))
    s, d, _, _ = synthetic.lidar_batch(2, 16384, seed0=44)
    src, dst = torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()
    with torch.no_grad():
        ref = engine.hregnet_forward(P, src, dst)
        with engine.chain_fork():
            out = engine.hregnet_forward(P, src, dst)
        torch.cuda.synchronize()
    for i in range(3):
        assert torch.equal(out["rotation"][i], ref["rotation"][i])
        assert torch.equal(out["translation"][i], ref["translation"][i])
    for key in ("desc_1", "desc_2", "desc_3", "xyz_3"):
        assert torch.equal(out["src_feats"][key], ref["src_feats"][key])


def test_graph_lanes_match_eager(net):
    """Two batches in flight (one stream each inside the graph): each lane's output
    is bitwise the eager forward of its own batch."""
    from pcd_reg_hregnet_amd import engine, synthetic
    P = net.prepared(torch.device("cuda"))
    data = [synthetic.lidar_batch(2, 4096, seed0=sd)[:2] for sd in (50, 51)]
    dev = [(torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()) for s, d in data]
    with torch.no_grad():
        gp = engine.GraphPipeline(P, dev[0][0], dev[0][1], lanes=2)
        gp.load(dev[1][0], dev[1][1], lane=1)
        refs = [engine.hregnet_forward(P, s, d) for s, d in dev]
        for steps in (1, 3):
            outs = gp.run(steps)
            torch.cuda.synchronize()
            for out, ref in zip(outs, refs):
                for i in range(3):
                    assert torch.equal(out["rotation"][i], ref["rotation"][i])
                    assert torch.equal(out["translation"][i], ref["translation"][i])
                assert torch.equal(out["src_feats"]["desc_3"], ref["src_feats"]["desc_3"])


def test_graph_merged_batches_match_eager(net):
    """The bench's HRegNet executor with reference batches merged per forward (bench --merge,
    engine.hregnet_forward sub_batch): two lanes, each forward running two batches of 2 pairs
    as one launch set, streamed rounds with and without front streaming -- every batch's outputs
    bitwise its own eager forward."""
    from pcd_reg_hregnet_amd import engine, synthetic
    P = net.prepared(torch.device("cuda"))
    data = [synthetic.lidar_batch(4, 4096, seed0=sd)[:2] for sd in (63, 64)]
    dev = [(torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()) for s, d in data]
    with torch.no_grad():
        gp = engine.GraphPipeline(P, dev[0][0], dev[0][1], lanes=2, sub_batch=2)
        gp.load(dev[1][0], dev[1][1], lane=1)
        refs = [[engine.hregnet_forward(P, s[i:i + 2], d[i:i + 2]) for i in (0, 2)] for s, d in dev]
        plan = [(2, False), (4, False), (2, True), (4, True)]  # (front streaming after prime())
        for n, front in plan:
            gp.prepare(n)
            if front:
                gp.prime()
                assert gp.fready is not None
            outs = gp.run_forwards(n, stream=True)
            torch.cuda.synchronize()
            for out, ref in zip(outs, refs):
                for k, r in enumerate(ref):
                    b = slice(2 * k, 2 * k + 2)
                    for i in range(3):
                        assert torch.equal(out["rotation"][i][b], r["rotation"][i])
                        assert torch.equal(out["translation"][i][b], r["translation"][i])
                    assert torch.equal(out["src_xyz_corres_1"][b], r["src_xyz_corres_1"])
                    assert torch.equal(out["src_feats"]["desc_3"][b], r["src_feats"]["desc_3"])


def test_graph_partial_round_matches_eager(net):
    """run_forwards(n) with n not a multiple of the lanes: full rounds, then a partial
    round on the first lanes; every lane's last output is bitwise its eager forward."""
    from pcd_reg_hregnet_amd import engine, synthetic
    P = net.prepared(torch.device("cuda"))
    data = [synthetic.lidar_batch(2, 4096, seed0=sd)[:2] for sd in (52, 53, 54)]
    dev = [(torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()) for s, d in data]
    with torch.no_grad():
        gp = engine.GraphPipeline(P, dev[0][0], dev[0][1], lanes=3)
        for ln in (1, 2):
            gp.load(dev[ln][0], dev[ln][1], lane=ln)
        refs = [engine.hregnet_forward(P, s, d) for s, d in dev]
        for n in (2, 4, 7):
            gp.prepare(n)
            outs = gp.run_forwards(n)
            torch.cuda.synchronize()
            assert len(outs) == 3
            for ln, out in enumerate(outs):
                if out is None:
                    continue
                for i in range(3):
                    assert torch.equal(out["rotation"][i], refs[ln]["rotation"][i]), (n, ln)
                    assert torch.equal(out["translation"][i], refs[ln]["translation"][i]), (n, ln)


def test_graph_streaming_matches_eager(net):
    """run_forwards(n, stream=True) (the bench's executor): each call's last replay also
    runs the next round's batched stage 1 and the next call starts from it.  Over calls of
    full and partial rounds every lane's output stays bitwise its eager forward, and
    load() discards the streamed stage 1 made from the old contents."""
    from pcd_reg_hregnet_amd import engine, synthetic
    P = net.prepared(torch.device("cuda"))
    data = [synthetic.lidar_batch(2, 4096, seed0=sd)[:2] for sd in (55, 56, 57, 58)]
    dev = [(torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()) for s, d in data]
    with torch.no_grad():
        gp = engine.GraphPipeline(P, dev[0][0], dev[0][1], lanes=3)
        assert gp.bs1
        for ln in (1, 2):
            gp.load(dev[ln][0], dev[ln][1], lane=ln)
        refs = [engine.hregnet_forward(P, s, d) for s, d in dev]

        def check(outs, want):
            torch.cuda.synchronize()
            for ln, out in enumerate(outs):
                if out is None:
                    continue
                for i in range(3):
                    assert torch.equal(out["rotation"][i], refs[want[ln]]["rotation"][i]), ln
                    assert torch.equal(out["translation"][i], refs[want[ln]]["translation"][i]), ln
                assert torch.equal(out["src_feats"]["desc_3"], refs[want[ln]]["src_feats"]["desc_3"])

        for n in (2, 3, 4, 7, 3):
            gp.prepare(n)
            outs = gp.run_forwards(n, stream=True)
            assert gp.ready is not None
            check(outs, [0, 1, 2])
        gp.load(dev[3][0], dev[3][1], lane=1)
        assert gp.ready is None
        check(gp.run_forwards(3, stream=True), [0, 3, 2])
        check(gp.run_forwards(3), [0, 3, 2])  # a non-streaming call after a streaming one
        assert gp.ready is None


def test_graph_front_streaming_matches_eager(net):
    """Front streaming (engine.FRONT_STREAM, the bench's executor after prime()): a round
    replays each lane's registration half of the batch whose feature extraction the previous
    round ran, beside the next batch's feature extraction.  Every lane's outputs stay bitwise
    its eager forward over several calls; a partial or non-streaming call falls back to the
    plain rounds; load() discards the pending fronts."""
    from pcd_reg_hregnet_amd import engine, synthetic
    P = net.prepared(torch.device("cuda"))
    data = [synthetic.lidar_batch(2, 4096, seed0=sd)[:2] for sd in (59, 60, 61, 62)]
    dev = [(torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()) for s, d in data]
    with torch.no_grad():
        gp = engine.GraphPipeline(P, dev[0][0], dev[0][1], lanes=3)
        assert gp.fs
        for ln in (1, 2):
            gp.load(dev[ln][0], dev[ln][1], lane=ln)
        refs = [engine.hregnet_forward(P, s, d) for s, d in dev]

        def check(outs, want):
            torch.cuda.synchronize()
            for ln, out in enumerate(outs):
                if out is None:
                    continue
                for i in range(3):
                    assert torch.equal(out["rotation"][i], refs[want[ln]]["rotation"][i]), ln
                    assert torch.equal(out["translation"][i], refs[want[ln]]["translation"][i]), ln
                    assert torch.equal(out["_fps_idx"][i], refs[want[ln]]["_fps_idx"][i]), ln
                for k in ("src_xyz_corres_1", "src_dst_weights_1", "src_xyz_corres_3"):
                    assert torch.equal(out[k], refs[want[ln]][k]), (ln, k)
                assert torch.equal(out["src_feats"]["desc_3"], refs[want[ln]]["src_feats"]["desc_3"])
                assert torch.equal(out["dst_feats"]["sigmas_1"], refs[want[ln]]["dst_feats"]["sigmas_1"])

        gp.run_forwards(2, stream=True)  # a partial round (the bench's warm-up shape)
        gp.prime()
        assert gp.fready is not None
        for n in (3, 6, 3):
            check(gp.run_forwards(n, stream=True), [0, 1, 2])
            assert gp.fready is not None
        gp.prepare(4)
        check(gp.run_forwards(4, stream=True), [0, 1, 2])  # partial: plain rounds
        assert gp.fready is None
        gp.prime()
        gp.load(dev[3][0], dev[3][1], lane=2)
        assert gp.fready is None and gp.ready is None
        gp.prime()
        check(gp.run_forwards(3, stream=True), [0, 1, 3])
        check(gp.run_forwards(3), [0, 1, 3])  # non-streaming after front streaming
        assert gp.fready is None


@pytest.mark.parametrize("lvl,split,pre,b6", [
    (0, False, False, False), (1, False, False, False), (2, False, False, False),
    (1, True, False, False), (2, True, False, False), (1, False, True, False),
    (2, False, True, False), (1, True, True, False), (2, True, True, False),
    (0, False, False, True), (1, False, False, True), (1, False, True, True),
    (1, True, False, True), (2, True, False, True), (1, True, True, True), (2, True, True, True)])
def test_fused_level_matches_layerwise(net, lvl, split, pre, b6, monkeypatch):
    """The fused level kernels (group_l1 / group_fused: activations in MFMA accumulators;
    group_split: channel-split through LDS; pre: the first convs' feature blocks
    precomputed per feature row, engine.LEVEL_PRE; b6: group_l1_6 / group_fused6, the
    products on the bf16 matrix cores at fp32 accuracy) against the layer-by-layer GEMM
    path on the same grouping; fp32 summation order differs, so within 1e-4."""
    from pcd_reg_hregnet_amd import engine, synthetic
    monkeypatch.setattr(engine, "LEVEL_PRE", pre)
    monkeypatch.setattr(engine, "B6_L1", b6)
    monkeypatch.setattr(engine, "B6_L2", b6)
    monkeypatch.setattr(engine, "B6_L3", b6)
    P = net.prepared(torch.device("cuda"))
    s, _, _, _ = synthetic.lidar_batch(2, 4096, seed0=60)
    pts = torch.from_numpy(s).cuda()
    with torch.no_grad():
        feats = w = None
        xyz = pts
        for level in range(lvl):
            kp, _, att, _, w, _ = engine.keypoint_level(P, level, xyz, feats, w)
            xyz, feats = kp, att
        grouped = engine.grouping(xyz, lvl, w)
        flag = ("FUSED_L1", "FUSED_L2", "FUSED_L3")[lvl]
        outs = []
        sflag = ("SPLIT_L2", "SPLIT_L3")[max(lvl, 1) - 1]
        old_split = getattr(engine, sflag)
        setattr(engine, sflag, split)
        for fused in (True, False):
            old = getattr(engine, flag)
            setattr(engine, flag, fused)
            try:
                outs.append(engine.keypoint_level(P, lvl, xyz, feats, w, grouped=grouped))
            finally:
                setattr(engine, flag, old)
                setattr(engine, sflag, old_split)
    torch.cuda.synchronize()
    (kp_f, sig_f, att_f, desc_f, w_f, _), (kp_r, sig_r, att_r, desc_r, w_r, _) = outs
    for a, b in ((kp_f, kp_r), (sig_f, sig_r), (att_f, att_r), (desc_f, desc_r)):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("G", [1, 7, 4099])
def test_l1_global_table_matches_lds_table(G):
    """hreg_group_l1_6g (weight table streamed from global memory, 4-wave workgroups) against
    hreg_group_l1_6 (table resident in LDS, 8-wave workgroups) on random tables and rows: the
    same arithmetic per group, so bitwise equal."""
    from pcd_reg_hregnet_amd import _lib
    L = _lib.load()
    rng = np.random.default_rng(G + 11)

    def t(x):
        return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).cuda()

    tb = t(rng.normal(0, 0.1, L.hreg_group_l1_6_table_floats()))
    geom, kx = t(rng.normal(size=(G * 64, 4))), t(rng.normal(size=(G * 64, 3)))
    outs = []
    for name in ("hreg_group_l1_6", "hreg_group_l1_6g"):
        kp = torch.full((G, 3), float("nan"), device="cuda")
        att = torch.full((G, 64), float("nan"), device="cuda")
        desc = torch.full((G, 64), float("nan"), device="cuda")
        _lib.call(name, tb, geom, kx, G, kp, att, desc, _lib.stream_handle())
        outs.append((kp, att, desc))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert not torch.isnan(b).any()
        assert torch.equal(a, b)


@pytest.mark.parametrize("pre,b6,split", [(True, True, True), (True, True, False), (True, False, False),
                                          (False, False, False)])
@pytest.mark.parametrize("name,C,N", [("fine_corres_1", 64, 1024), ("fine_corres_2", 128, 512)])
def test_fused_fine_head_matches_layerwise(net, name, C, N, pre, b6, split, monkeypatch):
    """group_head.hip (convs_1 + attention in one kernel; pre: descriptor blocks of
    convs_1[0] precomputed per point, engine.HEAD_PRE; b6: the bf16x6 kernel, products on
    the bf16 matrix cores at fp32 accuracy; split: coarse6.hip's channel-split kernel,
    hreg_corr_head6) against the GEMM + attend path."""
    from pcd_reg_hregnet_amd import engine
    monkeypatch.setattr(engine, "HEAD_PRE", pre)
    monkeypatch.setattr(engine, "B6_HEADS", b6)
    monkeypatch.setattr(engine, "SPLIT_FINE", split)
    P = net.prepared(torch.device("cuda"))
    g = torch.Generator().manual_seed(3)
    B = 2
    sx = (torch.rand(B, N, 3, generator=g) * 40 - 20).cuda()
    dx = (sx.cpu() + torch.randn(B, N, 3, generator=g) * 0.3).cuda()
    sd = torch.relu(torch.randn(B * N, C, generator=g)).cuda()
    dd = torch.relu(torch.randn(B * N, C, generator=g)).cuda()
    sw = torch.rand(B * N, generator=g).cuda()
    dw = torch.rand(B * N, generator=g).cuda()
    outs = []
    with torch.no_grad():
        for fused in (True, False):
            old = engine.FUSED_FINE
            engine.FUSED_FINE = fused
            try:
                outs.append(engine.fine_reg(P, name, B, sx, sd, dx, dd, sw, dw))
            finally:
                engine.FUSED_FINE = old
    torch.cuda.synchronize()
    (c_f, w_f), (c_r, w_r) = outs
    torch.testing.assert_close(c_f, c_r, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(w_f, w_r, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("B,b6,fused", [(1, False, False), (3, False, False), (3, True, False),
                                         (1, True, True), (3, True, True)])
def test_coarse_split_matches_concat_gemm(net, B, b6, fused, monkeypatch):
    """CoarseReg convs_1[0] as the 16-column GEMM + per-keypoint desc / knn_desc products
    added in the epilogue vs the one 528-deep GEMM over the concatenated rows
    (layers.py:364-384).  Only the fp32 summation order differs: 1e-4 on corres/weights."""
    from pcd_reg_hregnet_amd import engine
    monkeypatch.setattr(engine, "B6_GEMM", b6)
    monkeypatch.setattr(engine, "FUSED_COARSE", fused)
    P = net.prepared(torch.device("cuda"))
    g = torch.Generator().manual_seed(11 + B)
    N1, C = 256, 256
    xyz3 = (torch.rand(2 * B, N1, 3, generator=g) * 40 - 20).cuda()
    desc3 = torch.relu(torch.randn(2 * B * N1, C, generator=g)).cuda()
    sig3 = (torch.rand(2 * B * N1, generator=g) + 0.1).cuda()
    outs = []
    with torch.no_grad():
        for split in (True, False):
            old = engine.COARSE_SPLIT
            engine.COARSE_SPLIT = split
            try:
                outs.append(engine.coarse_reg(P, B, xyz3, desc3, sig3))
            finally:
                engine.COARSE_SPLIT = old
    torch.cuda.synchronize()
    (c_f, w_f), (c_r, w_r) = outs
    torch.testing.assert_close(c_f, c_r, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(w_f, w_r, rtol=1e-4, atol=1e-5)


def test_gemm_addends_vs_torch():
    """hreg_gemm's pre-epilogue addends (row_div and gather row sources) vs torch fp32."""
    from pcd_reg_hregnet_amd import engine
    rng = np.random.default_rng(7)
    R, N, K, k = 4096, 512, 16, 8
    A = rng.normal(size=(R, K)).astype(np.float32)
    W = (rng.normal(size=(N, K)) / 4).astype(np.float32)
    U = rng.normal(size=(R // k, N)).astype(np.float32)
    V = rng.normal(size=(300, N)).astype(np.float32)
    gi = rng.integers(0, 300, R).astype(np.int32)
    al = rng.uniform(0.5, 1.5, N).astype(np.float32)
    be = rng.normal(0, 0.1, N).astype(np.float32)
    t = {n: torch.from_numpy(v).cuda() for n, v in
         dict(A=A, W=W, U=U, V=V, gi=gi, al=al, be=be).items()}
    lin = engine.Lin(t["W"], t["al"], t["be"], True)
    out = engine.gemm([engine._seg(t["A"], 0, K)], lin, R,
                      adds=[engine._seg(t["U"], 0, 4, row_div=k),
                            engine._seg(t["V"], 0, 4, gather=t["gi"])]).cpu().numpy()
    pre = (A.astype(np.float64) @ W.T.astype(np.float64) + U[np.arange(R) // k] + V[gi])
    ref = np.maximum(pre * al + be, 0)
    scale = (np.abs(A) @ np.abs(W).T + np.abs(U[np.arange(R) // k]) + np.abs(V[gi])) * al + np.abs(be)
    assert np.all(np.abs(out - ref) <= 1e-5 * scale + 1e-6)


@pytest.mark.parametrize("pre,b6,split", [(True, True, True), (True, True, False), (True, False, False),
                                          (False, False, False)])
def test_fused_nbr_head_matches_layerwise(net, pre, b6, split, monkeypatch):
    """CoarseReg neighbour branch in one kernel (group_head.hip; pre: descriptor block of
    convs_2[0] precomputed per point; b6: bf16x6 products; split: coarse6.hip's
    channel-split kernel, hreg_nbr_head6s) vs GEMMs + attend."""
    from pcd_reg_hregnet_amd import engine
    monkeypatch.setattr(engine, "HEAD_PRE", pre)
    monkeypatch.setattr(engine, "B6_HEADS", b6)
    monkeypatch.setattr(engine, "SPLIT_NBR", split)
    P = net.prepared(torch.device("cuda"))
    g = torch.Generator().manual_seed(5)
    B, N1, C = 2, 256, 256
    xyz3 = (torch.rand(2 * B, N1, 3, generator=g) * 40 - 20).cuda()
    desc3 = torch.relu(torch.randn(2 * B * N1, C, generator=g)).cuda()
    sig3 = (torch.rand(2 * B * N1, generator=g) + 0.1).cuda()
    outs = []
    with torch.no_grad():
        for fused in (True, False):
            old = engine.FUSED_NBR
            engine.FUSED_NBR = fused
            try:
                outs.append(engine.coarse_reg(P, B, xyz3, desc3, sig3))
            finally:
                engine.FUSED_NBR = old
    torch.cuda.synchronize()
    (c_f, w_f), (c_r, w_r) = outs
    torch.testing.assert_close(c_f, c_r, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(w_f, w_r, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("G", [4, 12, 1024])
def test_nbr_head6_split_matches_chained(net, G):
    """hreg_nbr_head6s (channel-split, coarse6.hip) against hreg_nbr_head6 (register-chained,
    group_head.hip) on the prepared table and random rows: the same per-row arithmetic up
    to the accumulation of the three layers (both bf16x6, same chunk order), so the
    attention sums agree to fp32 rounding; 1e-5 relative."""
    from pcd_reg_hregnet_amd import _lib
    P = net.prepared(torch.device("cuda"))
    rng = np.random.default_rng(G)
    npts = G + 5
    desc = torch.from_numpy(np.abs(rng.normal(size=(npts, 256))).astype(np.float32)).cuda()
    pre = torch.from_numpy(rng.normal(size=(npts, 256)).astype(np.float32)).cuda()
    geom = torch.from_numpy(rng.normal(size=(G * 8, 4)).astype(np.float32)).cuda()
    gidx = torch.from_numpy(rng.integers(0, npts, G * 8).astype(np.int32)).cuda()
    outs = []
    for name in ("hreg_nbr_head6", "hreg_nbr_head6s"):
        out = torch.full((G, 256), float("nan"), device="cuda")
        _lib.call(name, P.nbr_table6, desc, gidx, geom, G, out, pre, _lib.stream_handle())
        outs.append(out)
    torch.cuda.synchronize()
    assert not torch.isnan(outs[1]).any()
    torch.testing.assert_close(outs[1], outs[0], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("key,C,rows,mode", [(("det", 0), 64, 1024, 0), (("det", 1), 128, 512, 0),
                                           (("det", 2), 256, 256, 0), ("coarse", 512, 256, 1),
                                           ("fine_corres_2", 256, 512, 1),
                                           ("fine_corres_1", 128, 1024, 1),
                                           # ragged: row-tile counts not a multiple of the
                                           # head's row tiles per workgroup (HREG_HEAD_JT)
                                           ("coarse", 512, 96, 1), ("fine_corres_1", 128, 160, 1)])
@pytest.mark.parametrize("b6", [False, True])
def test_fused_mlp_head_matches_layerwise(net, key, C, rows, mode, b6, monkeypatch):
    """mlp_head.hip (mlp1 -> mlp2 -> mlp3 + softplus/sigmoid in one launch; b6: bf16x6
    products) against two GEMMs + hreg_head_out; fp32 summation order differs, so within
    1e-4 (and the per-cloud sigma -> weight normalisation, models.py:30-32)."""
    from pcd_reg_hregnet_amd import _lib, engine
    monkeypatch.setattr(engine, "B6_MLP", b6)
    P = net.prepared(torch.device("cuda"))
    g = torch.Generator().manual_seed(7)
    nclouds = 3
    x = torch.relu(torch.randn(nclouds * rows, C, generator=g)).cuda()
    outs = []
    with torch.no_grad():
        for fused in (True, False):
            old = engine.FUSED_HEAD
            engine.FUSED_HEAD = fused
            try:
                outs.append(engine.mlp_head(P, key, x, nclouds, rows, mode, want_weights=mode == 0))
            finally:
                engine.FUSED_HEAD = old
    torch.cuda.synchronize()
    (o_f, w_f), (o_r, w_r) = outs
    torch.testing.assert_close(o_f, o_r, rtol=1e-4, atol=1e-6)
    if mode == _lib.HREG_HEAD_SOFTPLUS:
        torch.testing.assert_close(w_f, w_r, rtol=1e-4, atol=1e-6)
    # one pair's rows give the same bits alone as inside the batch
    with torch.no_grad():
        one, _ = engine.mlp_head(P, key, x[rows:2 * rows].contiguous(), 1, rows, mode)
    assert torch.equal(one, o_f[rows:2 * rows])


def test_mlp_head_rejects_bad_shapes(net):
    from pcd_reg_hregnet_amd import _lib
    P = net.prepared(torch.device("cuda"))
    x = torch.zeros(64, 96, device="cuda")
    out = torch.empty(64, device="cuda")
    with pytest.raises(RuntimeError, match="unsupported"):
        _lib.call("hreg_mlp_head", P.head_table["coarse"], 96, x, 96, 1, 64, 0, out, None,
                  _lib.stream_handle())
    with pytest.raises(RuntimeError, match="unsupported"):
        _lib.call("hreg_mlp_head", P.head_table["coarse"], 64, x, 96, 1, 48, 0, out, None,
                  _lib.stream_handle())


@pytest.fixture(scope="module")
def net_v2():
    from helpers import state_dict_v2_torch
    from pcd_reg_hregnet_amd.models import Model_V2
    m = Model_V2(Args())
    m.load_state_dict(state_dict_v2_torch())
    return m.cuda().eval()


@pytest.mark.parametrize("fixture", ["model_v2_lidar_b2_n4096.npz",
                                     "model_v2_lidar_b1_n65536.npz",
                                     "model_v2_lidar_b2_n65536.npz"])
def test_model_v2_matches_reference_fixture(net_v2, fixture):
    """Model_V2 against the reference's own run of the same
    weights/inputs; torch's generator is seeded as the fixture run was, so the
    randperm "prime" shuffles are the same draws.  The N=65536 cases are config 5's
    cloud size (level-1 FPS on the multi-workgroup cluster kernel, spatially indexed
    level-1 grouping); at B=2 the fixture's seed makes both prime shuffles the swap
    (model_v2/layers.py:492,497), so the batch permutation is exercised at that size."""
    from test_oracle_golden import compare_v2
    from pcd_reg_hregnet_amd import engine
    g = load_npz(fixture)
    B = g["src"].shape[0]
    P = net_v2.prepared(torch.device("cuda"))
    torch.manual_seed(int(g["perm_seed"]))
    engine.INDEX_RECORD = {}
    try:
        with torch.no_grad():
            r = engine.model_v2_forward(P, torch.from_numpy(g["src"]).cuda(),
                                        torch.from_numpy(g["dst"]).cuda())
        torch.cuda.synchronize()
        r["_knn"] = engine.INDEX_RECORD
    finally:
        engine.INDEX_RECORD = None

    def cpu(x):
        if isinstance(x, torch.Tensor):
            return x.cpu().numpy()
        if isinstance(x, list):
            return [cpu(v) for v in x]
        if isinstance(x, dict):
            return {k: cpu(v) for k, v in x.items()}
        return x
    r = cpu(r)
    np.testing.assert_array_equal(r["_fps_idx"][0][:B], g["src_fps_1"])
    np.testing.assert_array_equal(r["_fps_idx"][0][B:], g["dst_fps_1"])
    compare_v2(r, g, title="GPU vs " + fixture)
    if fixture == "model_v2_lidar_b2_n65536.npz":  # the shuffle is the swap, not the identity
        np.testing.assert_array_equal(g["src_dst_weights_2_prime"][0], g["src_dst_weights_2"][1])
        np.testing.assert_array_equal(r["src_dst_weights_2_prime"][0], r["src_dst_weights_2"][1])


def test_model_v2_module_api(net_v2):
    """Model_V2.forward returns the reference's dict (model_v2/models.py:170-183)."""
    g = load_npz("model_v2_lidar_b2_n4096.npz")
    torch.manual_seed(int(g["perm_seed"]))
    with torch.no_grad():
        r = net_v2(torch.from_numpy(g["src"]).cuda(), torch.from_numpy(g["dst"]).cuda())
    assert "_fps_idx" not in r
    assert tuple(r["src_dst_feats_2"].shape) == (2, 128, 512)
    assert tuple(r["src_dst_weights_2_prime"].shape) == (2, 512)
    assert tuple(r["src_xyz_2_trans"].shape) == (2, 512, 3)
    np.testing.assert_allclose(r["rotation"][-1].cpu().numpy(), g["R1"], atol=1e-4)
    np.testing.assert_allclose(r["translation"][-1].cpu().numpy(), g["t1"], atol=1e-4)


@pytest.mark.parametrize("batched", [False, True])
def test_model_v2_graph_pipeline_matches_eager(net_v2, batched):
    """Model_V2 through the graph executor (2 lanes, N=65536 level-1 on the side streams, or
    batched: one bounded-concurrency cluster-FPS launch over both lanes' clouds,
    engine.V2_BATCH_STAGE1): outputs bitwise those of the eager forward, prime shuffles drawn
    from the host generator per round exactly as the eager forward draws them."""
    from pcd_reg_hregnet_amd import engine
    g = load_npz("model_v2_lidar_b1_n65536.npz")
    P = net_v2.prepared(torch.device("cuda"))
    src = torch.from_numpy(g["src"]).cuda()
    dst = torch.from_numpy(g["dst"]).cuda()
    old = engine.V2_BATCH_STAGE1
    try:
        engine.V2_BATCH_STAGE1 = batched
        with torch.no_grad():
            gp = engine.GraphPipeline(P, src, dst, lanes=2, v2=True)
            assert gp.bs1 == batched
            torch.manual_seed(int(g["perm_seed"]))
            outs = gp.run(1)
            torch.manual_seed(int(g["perm_seed"]))
            ref = engine.model_v2_forward(P, src, dst)
    finally:
        engine.V2_BATCH_STAGE1 = old
    torch.cuda.synchronize()
    for o in outs[:1]:
        for key in ("src_dst_feats_2", "src_dst_feats_2_prime", "src_dst_weights_2",
                    "src_dst_weights_2_prime", "src_xyz_2_trans"):
            assert torch.equal(o[key], ref[key]), key
        for i in range(3):
            assert torch.equal(o["rotation"][i], ref["rotation"][i])
            assert torch.equal(o["translation"][i], ref["translation"][i])
    np.testing.assert_allclose(outs[1]["rotation"][-1].cpu().numpy(), g["R1"], atol=1e-4)


def test_b6_kernels_deterministic(net):
    """The bf16x6 kernels (group_l1_6, group_fused6, fine_head6 / nbr_head6) give the same
    bits run after run with two workgroups per CU (two waves per SIMD): the configuration
    in which packed-fp32 VALU ops next to the bf16 MFMAs gave nondeterministic wrong values
    (build.NO_PACKED_F32); and level 1 matches the fp32-MFMA kernel at 1e-4."""
    from pcd_reg_hregnet_amd import engine, synthetic
    P = net.prepared(torch.device("cuda"))
    s, d, _, _ = synthetic.lidar_batch(4, 8192, seed0=70)
    src, dst = torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()
    with torch.no_grad():
        runs = [engine.hregnet_forward(P, src, dst) for _ in range(4)]
        g = engine.grouping(src, 0, None)
        old = engine.B6_L1
        try:
            engine.B6_L1 = False
            ref = engine.keypoint_level(P, 0, src, None, None, grouped=g)
            engine.B6_L1 = True
            b6 = engine.keypoint_level(P, 0, src, None, None, grouped=g)
        finally:
            engine.B6_L1 = old
    torch.cuda.synchronize()
    for r in runs[1:]:
        for key in ("desc_1", "desc_2", "desc_3", "xyz_1", "xyz_2", "xyz_3"):
            assert torch.equal(r["src_feats"][key], runs[0]["src_feats"][key]), key
        for i in range(3):
            assert torch.equal(r["rotation"][i], runs[0]["rotation"][i])
        assert torch.equal(r["src_dst_weights_1"], runs[0]["src_dst_weights_1"])
    for a, b in zip(ref[:4], b6[:4]):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("G", [4096, 4094, 4090, 2])
def test_level3_two_tile_kernel_bitwise(net, G):
    """hreg_group_split6j_l3 (two 32-row tiles per wave sharing every weight piece)
    gives hreg_group_split6_l3's bits -- keypoints, attentive features, descriptors --
    including tile counts that leave the last set short (G = 4094, 4090: its missing tiles
    recompute the last tile) and a single tile."""
    from pcd_reg_hregnet_amd import _lib, engine
    P = net.prepared(torch.device("cuda"))
    g = torch.Generator(device="cpu").manual_seed(G)
    K, C, nrows = 16, 128, 2 * G
    R = G * K
    geom = torch.randn(R, 4, generator=g).cuda()
    kx = torch.randn(R, 3, generator=g).cuda()
    gidx = torch.randint(0, nrows, (R,), generator=g, dtype=torch.int32).cuda()
    feats = torch.rand(nrows, C, generator=g).cuda()
    pre = engine.gemm([engine._seg(feats, 0, C)], P.level_pre6[2], nrows)
    outs = []
    for name in ("hreg_group_split6_l3", "hreg_group_split6j_l3"):
        kp = torch.empty(G, 3, device="cuda")
        att = torch.empty(G, 256, device="cuda")
        desc = torch.empty(G, 256, device="cuda")
        _lib.call(name, P.l3s_table6, geom, kx, gidx, feats, G, kp, att, desc, pre, _lib.stream_handle())
        outs.append((kp, att, desc))
    torch.cuda.synchronize()
    for a, b, nm in zip(outs[0], outs[1], ("kp", "att_feat", "desc")):
        assert torch.equal(a, b), nm


def test_heads_two_tile_bitwise(net):
    """The FineReg heads (N1 = 256 / 128) and the neighbour branch on two 32-row tiles per
    workgroup (hreg_corr_head6x / hreg_nbr_head6sx, row_tiles 2: the default) give the
    one-tile kernels' bits: the whole forward compared with engine.HEAD_ROW_TILES = 1."""
    from pcd_reg_hregnet_amd import engine, synthetic
    P = net.prepared(torch.device("cuda"))
    s, d, _, _ = synthetic.lidar_batch(3, 16384, seed0=91)
    src, dst = torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()
    outs = []
    old = engine.HEAD_ROW_TILES
    try:
        for rt in (1, 0):
            engine.HEAD_ROW_TILES = rt
            with torch.no_grad():
                outs.append(engine.hregnet_forward(P, src, dst))
    finally:
        engine.HEAD_ROW_TILES = old
    torch.cuda.synchronize()
    a, b = outs
    for key in a:
        if isinstance(a[key], torch.Tensor):
            assert torch.equal(a[key], b[key]), key
    for i in range(3):
        assert torch.equal(a["rotation"][i], b["rotation"][i])
        assert torch.equal(a["translation"][i], b["translation"][i])


def test_grouped_head_gemms_bitwise(net):
    """engine.GROUPED_HEAD_GEMMS: the heads' precomputed blocks and the original cosine
    similarity from one hreg_gemm_grouped launch give the same bits as their five separate
    hreg_gemm launches (every output of the forward)."""
    from pcd_reg_hregnet_amd import engine, synthetic
    s, d, _, _ = synthetic.lidar_batch(3, 4096, seed0=77)
    old = engine.GROUPED_HEAD_GEMMS
    try:
        engine.GROUPED_HEAD_GEMMS = True
        a = _run(net, s, d)
        engine.GROUPED_HEAD_GEMMS = False
        b = _run(net, s, d)
    finally:
        engine.GROUPED_HEAD_GEMMS = old
    for key in ("src_xyz_corres_3", "src_xyz_corres_2", "src_xyz_corres_1", "src_dst_weights_3",
                "src_dst_weights_2", "src_dst_weights_1"):
        np.testing.assert_array_equal(a[key], b[key], key)
    for i in range(3):
        np.testing.assert_array_equal(a["rotation"][i], b["rotation"][i])
        np.testing.assert_array_equal(a["translation"][i], b["translation"][i])


def test_model_v2_merged_batches_match_separate_forwards(net_v2):
    """engine.hregnet_forward(sub_batch=2) over 3 reference batches of 2 pairs merged into one
    launch set (the bench's Model_V2 executor, --merge): every output of every batch bitwise that
    of the batch's own forward, including the prime copies -- shuffled within each batch, the
    draws in batch order as three separate forwards draw them -- and the weighted SVD's identity
    fallback applies per batch (a non-finite pair resets its own batch only)."""
    from pcd_reg_hregnet_amd import engine, synthetic
    P = net_v2.prepared(torch.device("cuda"))
    s, d, _, _ = synthetic.lidar_batch(6, 8192, seed0=31)
    src, dst = torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()
    with torch.no_grad():
        torch.manual_seed(7)
        merged = engine.model_v2_finish(engine.hregnet_forward(P, src, dst, v2=True, sub_batch=2), 2)
        torch.manual_seed(7)
        sep = [engine.model_v2_forward(P, src[i:i + 2], dst[i:i + 2]) for i in (0, 2, 4)]
    torch.cuda.synchronize()
    for j, o in enumerate(sep):
        b = slice(2 * j, 2 * j + 2)
        for key in ("src_dst_feats_2", "src_dst_feats_2_prime", "src_dst_weights_2",
                    "src_dst_weights_2_prime", "src_xyz_2_trans", "src_xyz_corres_1"):
            assert torch.equal(merged[key][b], o[key]), (j, key)
        for i in range(3):
            assert torch.equal(merged["rotation"][i][b], o["rotation"][i]), (j, i)
            assert torch.equal(merged["translation"][i][b], o["translation"][i]), (j, i)
    # the identity fallback of layers.py:485-493 per batch: pair 3 (batch 1) has no weight
    x = torch.randn(6, 64, 3, device="cuda")
    a = 0.3
    Rz = torch.tensor([[math.cos(a), -math.sin(a), 0.0], [math.sin(a), math.cos(a), 0.0], [0.0, 0.0, 1.0]],
                      device="cuda")
    c = x @ Rz.T + 0.01
    w = torch.rand(6, 64, device="cuda") + 0.1
    w[3] = float("nan")
    R_, t_, _, _ = engine.weighted_svd(x, c, w, group=2)
    eye = torch.eye(3, device="cuda")
    assert torch.equal(R_[2], eye) and torch.equal(R_[3], eye)
    for i in (0, 1, 4, 5):
        assert not torch.equal(R_[i], eye) and torch.isfinite(R_[i]).all()
    R1_, _, _, _ = engine.weighted_svd(x, c, w)  # one batch of 6: all reset
    assert all(torch.equal(R1_[i], eye) for i in range(6))

@pytest.mark.gpu
@pytest.mark.parametrize("key", [("det", 0), ("det", 1), ("det", 2), "coarse"])
def test_mlp_head_row_tiles(net, key):
    """hreg_mlp_head6x with one 32-row tile per workgroup (chain_fork's single-forward form) vs
    the default 2-4 tiles per workgroup: the same bits, sigma / weight outputs and the per-cloud
    weights alike, with a tile count that leaves the last workgroup's group partial."""
    from pcd_reg_hregnet_amd import _lib
    P = net.prepared(torch.device("cuda"))
    C = {("det", 0): 64, ("det", 1): 128, ("det", 2): 256, "coarse": 512}[key]
    nclouds, rows = 3, 96  # 9 tiles of 32 rows
    g = torch.Generator(device="cpu").manual_seed(C)
    x = torch.randn(nclouds * rows, C, generator=g).cuda()
    mode = _lib.HREG_HEAD_SOFTPLUS if key != "coarse" else _lib.HREG_HEAD_SIGMOID
    res = []
    for rt in (0, 1):
        out = torch.full((nclouds * rows,), float("nan"), device="cuda")
        w = torch.full((nclouds * rows,), float("nan"), device="cuda") if key != "coarse" else None
        _lib.call("hreg_mlp_head6x", P.head_table6[key], C, x, C, nclouds, rows, mode, out, w, rt,
                  _lib.stream_handle())
        res.append((out, w))
    torch.cuda.synchronize()
    assert not torch.isnan(res[0][0]).any()
    assert torch.equal(res[0][0], res[1][0])
    if key != "coarse":
        assert torch.equal(res[0][1], res[1][1])



@pytest.mark.parametrize("G", [2048, 2044])
def test_coarse_head_row_tiles(net, G):
    """hreg_corr_head6x at N1 = 512 (CoarseReg): the one-tile kernel fills every output (also for
    a partial last row tile), and the two-tile form -- measured slower (r5) and removed -- is
    refused as unsupported instead of computing something else."""
    from pcd_reg_hregnet_amd import _lib
    P = net.prepared(torch.device("cuda"))
    g = torch.Generator(device="cpu").manual_seed(G)
    R = G * 8
    small = torch.randn(R, 16, generator=g).cuda()
    ud0 = torch.randn(G, 512, generator=g).cuda()
    ud1 = torch.randn(G, 512, generator=g).cuda()
    gidx = torch.randint(0, G, (R,), generator=g, dtype=torch.int32).cuda()
    kx = torch.randn(R, 3, generator=g).cuda()
    corres = torch.full((G, 3), float("nan"), device="cuda")
    att = torch.full((G, 512), float("nan"), device="cuda")
    _lib.call("hreg_corr_head6x", P.coarse_table6, 512, small, ud0, ud1, gidx, kx, G, corres, att, 1,
              _lib.stream_handle())
    torch.cuda.synchronize()
    assert not torch.isnan(corres).any() and not torch.isnan(att).any()
    with pytest.raises(RuntimeError, match="(?i)unsupported"):
        _lib.call("hreg_corr_head6x", P.coarse_table6, 512, small, ud0, ud1, gidx, kx, G, corres, att, 2,
                  _lib.stream_handle())


@pytest.mark.parametrize("use_sim,use_neighbor", [(True, True), (True, False), (False, True), (False, False)])
def test_coarse_reg_variants_vs_oracle(net, use_sim, use_neighbor):
    """CoarseReg(use_sim, use_neighbor) alone in eval mode (layers.py:237-244,
    290, 315, 368-379) against the oracle's restatement of every variant, on the network's own
    level-3 keypoints and descriptors of a LiDAR pair: the same descriptor-space and neighbour
    kNN selections (canonical order), correspondences within the R/t bar and weights within
    1e-5.  The variant's weights are the trained head's with the absent features' columns
    dropped."""
    from oracle import oracle
    from pcd_reg_hregnet_amd import models, synthetic
    s, d, _, _ = synthetic.lidar_batch(2, 16384, seed0=31)
    with torch.no_grad():
        out = net(torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda())
    sx, sdsc = out["src_feats"]["xyz_3"], out["src_feats"]["desc_3"]
    dx, ddsc = out["dst_feats"]["xyz_3"], out["dst_feats"]["desc_3"]
    B, N = sx.shape[:2]
    g = torch.Generator().manual_seed(3)
    sw = (0.5 + torch.rand(B, N, generator=g)).cuda()
    dw = (0.5 + torch.rand(B, N, generator=g)).cuda()
    m = models.CoarseReg(8, 256, use_sim, use_neighbor).cuda().eval()
    ref = net.coarse_corres.state_dict()
    keep = list(range(524)) + ([524, 525] if use_sim else []) + ([526, 527] if use_neighbor else [])
    sd = dict(ref)
    sd["convs_1.0.weight"] = ref["convs_1.0.weight"][:, keep].contiguous()
    m.load_state_dict(sd)
    corres, w = m(sx, sdsc, dx, ddsc, sw, dw)
    torch.cuda.synchronize()
    npsd = {"c." + k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    oc, ow, _ = oracle.coarse_reg(npsd, "c", sx.cpu().numpy(), sdsc.cpu().numpy(), dx.cpu().numpy(),
                                  ddsc.cpu().numpy(), sw.cpu().numpy(), dw.cpu().numpy(),
                                  use_sim=use_sim, use_neighbor=use_neighbor)
    np.testing.assert_allclose(corres.cpu().numpy(), oc, rtol=0, atol=1e-4)
    np.testing.assert_allclose(w.cpu().numpy(), ow, rtol=0, atol=1e-5)
    if use_sim and use_neighbor:  # the module alone == the head inside HRegNet's forward
        full = net.prepared(torch.device("cuda"))
        from pcd_reg_hregnet_amd import engine
        with torch.no_grad():
            c2, w2 = engine.coarse_reg(full, B, torch.cat([sx, dx]).contiguous(),
                                       torch.cat([sdsc, ddsc]).transpose(1, 2).reshape(2 * B * N, -1).contiguous(),
                                       torch.cat([sw, dw]).reshape(-1).contiguous())
        assert torch.equal(c2, corres) and torch.equal(w2, w)
