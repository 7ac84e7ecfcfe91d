"""Pins the CPU oracle (oracle/) against the reference-generated fixtures.

The fixtures were produced by tests/golden/make_golden.py from the reference's
own Python model with a literal emulation of its CUDA FPS kernel; see that
script's header.  Index outputs must match bit-exactly; floating outputs
within the stated tolerances.
"""
import numpy as np
import pytest

import parity
from helpers import load_npz, state_dict_numpy, state_dict_v2_torch, v2_perms
from oracle import oracle

OPS = load_npz("ops.npz")
FPS_CASES = sorted({k[4:-4] for k in OPS if k.startswith("fps_") and k.endswith("_idx")})
KNN_CASES = sorted({k[4:-4] for k in OPS if k.startswith("knn_") and k.endswith("_idx")})


def test_opt_n_threads():
    # cuda_utils.h:22-26 (double log, truncated)
    for n, bs in [(1, 1), (3, 2), (100, 64), (512, 512), (1000, 512), (1023, 512),
                  (1024, 1024), (16384, 1024), (65536, 1024)]:
        assert oracle.opt_n_threads(n) == bs


@pytest.mark.parametrize("case", FPS_CASES)
def test_fps_bit_exact(case):
    xyz = OPS[f"fps_{case}_xyz"]
    m = int(OPS[f"fps_{case}_m"])
    w = OPS.get(f"fps_{case}_w")
    got = oracle.fps(xyz, m, w)
    np.testing.assert_array_equal(got, OPS[f"fps_{case}_idx"])


@pytest.mark.parametrize("case", KNN_CASES)
def test_knn_bit_exact(case):
    p1, p2 = OPS[f"knn_{case}_p1"], OPS[f"knn_{case}_p2"]
    K = OPS[f"knn_{case}_idx"].shape[-1]
    d, i = oracle.knn(p1, p2, K)
    np.testing.assert_array_equal(i, OPS[f"knn_{case}_idx"])
    np.testing.assert_array_equal(d, OPS[f"knn_{case}_dist"])


def test_gather_points_roundtrip():
    rng = np.random.default_rng(0)
    pts = rng.normal(size=(2, 5, 300)).astype(np.float32)
    idx = rng.integers(0, 300, (2, 40)).astype(np.int32)
    out = oracle.gather_points(pts, idx)
    np.testing.assert_array_equal(out, np.take_along_axis(pts, idx[:, None, :].repeat(5, 1), 2))
    g = oracle.gather_points_grad(np.ones_like(out), idx, 300)
    cnt = np.zeros((2, 300))
    for b in range(2):
        np.add.at(cnt[b], idx[b], 1)
    np.testing.assert_array_equal(g[:, 0], cnt)


@pytest.fixture(scope="module")
def sd():
    return state_dict_numpy()


def compare_forward(r, g, title=""):
    """The end-to-end parity contract (tests/parity.py): level-1 FPS bit-exact, every
    other selection the reference's unless it is a float64 near tie (or downstream of
    one), every continuous output on the rows with identical selections within 1e-5
    normalised, R/t within 1e-4.  r: an engine / oracle result; g: a fixture-layout dict.
    Prints the observed numbers and returns them."""
    return parity.check(parity.as_layout(r, g["src"].shape[0]), g, title)


@pytest.mark.parametrize("fixture", ["hregnet_lidar_b2_n4096.npz", "hregnet_cube_b1_n16384.npz"])
def test_forward_matches_reference(sd, fixture):
    g = load_npz(fixture)
    r = oracle.hregnet_forward(sd, g["src"], g["dst"])
    # FPS indices: level 1 depends only on the input -> exact
    np.testing.assert_array_equal(r["src_feats"]["fps_idx_1"], g["src_fps_1"])
    np.testing.assert_array_equal(r["dst_feats"]["fps_idx_1"], g["dst_fps_1"])
    compare_forward(r, g, title="oracle vs " + fixture)


def test_random_sampling_forward_matches_reference(sd):
    """use_fps=False (layers.py:144-147): the oracle fed the reference's own random samples
    (hregnet_randsample_b2_n4096.npz) against the reference's forward."""
    g = load_npz("hregnet_randsample_b2_n4096.npz")
    samples = [g[f"{p}_fps_{lv}"] for p in ("src", "dst") for lv in (1, 2, 3)]
    r = oracle.hregnet_forward(sd, g["src"], g["dst"], samples=samples)
    compare_forward(r, g, title="oracle vs hregnet_randsample_b2_n4096.npz")


def test_random_sample_draws_match_reference():
    """engine.random_samples draws torch.randperm(N)[:M] per level on the host generator
    in the reference's order (src levels 1-3, then dst), one draw per cloud set: after the
    fixture's seed it reproduces the reference's samples exactly (no GPU needed)."""
    import torch
    from pcd_reg_hregnet_amd import engine
    g = load_npz("hregnet_randsample_b2_n4096.npz")
    B, N = g["src"].shape[:2]
    torch.manual_seed(int(g["perm_seed"]))
    got = engine.random_samples(2, B, engine.level_input_sizes(N), "cpu")
    for lv in (1, 2, 3):
        want = np.concatenate([g[f"src_fps_{lv}"], g[f"dst_fps_{lv}"]], 0)
        np.testing.assert_array_equal(got[lv - 1].numpy(), want)


def compare_v2(r, g, title=""):
    """Model_V2 parity (model_v2/models.py:170-183): the HRegNet contract of
    compare_forward on its shared outputs, then the Model_V2 extras (the transformed level-2
    keypoints, FineReg2's mlpx features and weights, their prime copies) on the rows with
    identical selections within the same 1e-5, and the prime copies exactly the batch
    permutation of their originals."""
    B = g["src"].shape[0]
    ours = parity.as_layout(r, B)
    ref = dict(g)
    for lv in (1, 2, 3):
        ref[f"corres_{lv}"] = g[f"src_xyz_corres_{lv}"]
    ref["weights_2"] = g["src_dst_weights_2"]
    st, bad = parity.evaluate(ours, ref)
    ok = ~st.pop("_affected_heads_2")
    for key, q in (("src_xyz_2_trans", "xyz_2"), ("src_dst_feats_2", "dst_feats_2"),
                   ("src_dst_weights_2", "weights_2")):
        a, b = np.asarray(r[key]), g[key + "_64"]
        if key == "src_dst_feats_2":
            a, b = a.transpose(0, 2, 1), b.transpose(0, 2, 1)
        st[key + "_vs_f64"] = e = parity.nerr(a[ok], b[ok])
        if e > parity.feat_bar(q):
            bad.append(f"{key}: {e:.2e} > bar {parity.feat_bar(q):.2e}")
    parity.report(st, title, bad)
    assert not bad, "\n".join(bad)
    a = np.asarray(r["dst_xyz_2"])
    assert np.array_equal(a, np.asarray(r["dst_feats"]["xyz_2"]))
    for key, base in (("src_dst_feats_2_prime", "src_dst_feats_2"),
                      ("src_dst_weights_2_prime", "src_dst_weights_2")):
        for d in (r, g):  # the same batch permutation as the reference's own draw
            perm = [int(np.nonzero([np.array_equal(np.asarray(d[key])[i], np.asarray(d[base])[j])
                                    for j in range(B)])[0][0]) for i in range(B)]
            assert sorted(perm) == list(range(B)), key
            if d is r:
                ours_perm = perm
        assert perm == ours_perm, key
    return st


@pytest.mark.parametrize("fixture", ["model_v2_lidar_b2_n4096.npz",
                                     "model_v2_lidar_b1_n65536.npz",
                                     "model_v2_lidar_b2_n65536.npz"])
def test_model_v2_matches_reference(fixture):
    """oracle.model_v2_forward vs the reference Model_V2 run (make_golden.py)."""
    g = load_npz(fixture)
    sd = {k: v.numpy() for k, v in state_dict_v2_torch().items()}
    pf, pw = v2_perms(g["perm_seed"], g["src"].shape[0])
    r = oracle.model_v2_forward(sd, g["src"], g["dst"], pf, pw)
    np.testing.assert_array_equal(r["src_feats"]["fps_idx_1"], g["src_fps_1"])
    compare_v2(r, g, title="oracle vs " + fixture)


LOSS = load_npz("transformation_loss.npz")
LOSS_NAMES = ("loss", "loss_R", "loss_t", "R_err", "geodesic_dist", "T_err", "eucl_dist")


def check_loss(res, c, i):
    """Tolerances: 1e-5 relative on the means/Euler angles/RTE; the geodesic (RRE) is
    acos near 1 for small errors -- an fp32 ulp of the trace moves it by ~0.03 deg --
    so it is compared with atol 0.05 deg."""
    for k, name in enumerate(LOSS_NAMES):
        want = LOSS[f"c{c}_{name}"][i]
        atol = 5e-2 if name == "geodesic_dist" else 1e-5
        np.testing.assert_allclose(np.asarray(res[k]), want, rtol=1e-5, atol=atol, err_msg=name)


@pytest.mark.parametrize("c", range(int(LOSS["ncases"])))
def test_transformation_loss_matches_reference(c):
    """oracle.transformation_loss vs the reference losses.py:97-164 run (make_golden.py)."""
    for i in range(LOSS[f"c{c}_pred_R"].shape[0]):
        res = oracle.transformation_loss(LOSS[f"c{c}_pred_R"][i], LOSS[f"c{c}_pred_t"][i],
                                         LOSS[f"c{c}_gt_R"][i], LOSS[f"c{c}_gt_t"][i],
                                         alpha=float(LOSS["alpha"]))
        check_loss(res, c, i)


def test_euler_xyz_matches_scipy():
    """The restated pytorch3d matrix_to_euler_angles("XYZ") is scipy's intrinsic 'XYZ'
    on rotation matrices (an independent pin for the absent pytorch3d)."""
    from scipy.spatial.transform import Rotation
    R = Rotation.random(64, random_state=5).as_matrix()
    z = np.zeros((64, 3))
    res = oracle.transformation_loss(np.eye(3)[None].repeat(64, 0), z, R, z)
    want = np.mean(np.abs(Rotation.from_matrix(R).as_euler("XYZ", degrees=True)), axis=0)
    np.testing.assert_allclose(res[3], want, rtol=1e-4)
