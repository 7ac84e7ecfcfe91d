"""Data side in front of the path on the GPU against fixtures the
reference itself produced (tests/golden/make_golden.py --perturb-only:
transform/rodrigues.py, transform/dataset_transforms.py, dataset/dataset_utils.py).

Bars: the range filter and the resampler are index/copy work -> bit-exact.  The SE(3)
algebra is float32 with device libm sin/cos/acos/tan (not torch's CPU libm), so the
values agree to a few ulp: exp 1e-6, log 1e-5 away from t = pi; near t = pi the log is
ill-conditioned (w = (R - R^T) / (2 sinc1(t)), sinc1 -> 0): there w may move by 5e-4
(the reference's own float32 log does not round-trip there either: exp(log(g)) is off
by up to 0.29 in its own outputs), and exp(log(g)) = g is required (1e-5) away from pi.
"""
import numpy as np
import pytest
import torch

from helpers import load_npz

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g():
    return load_npz("perturb.npz")


def cu(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def test_se3_exp_log(g):
    from pcd_reg_hregnet_amd.perturb import SE3
    x = g["se3_x"]
    ang = np.linalg.norm(x[:, :3], axis=1)
    G = SE3.exp(cu(x))
    np.testing.assert_allclose(G.cpu().numpy(), g["se3_exp"], atol=1e-6, rtol=0)
    L = SE3.log(cu(g["se3_exp"])).cpu().numpy()
    generic = ang < 3.0
    np.testing.assert_allclose(L[generic], g["se3_log"][generic], atol=1e-5, rtol=0)
    np.testing.assert_allclose(L[~generic], g["se3_log"][~generic], atol=5e-4, rtol=0)
    back = SE3.exp(cu(L[generic])).cpu().numpy()
    np.testing.assert_allclose(back, g["se3_exp"][generic], atol=1e-5, rtol=0)


def test_so3_log_pi_branch(g):
    """Exact pi rotations take the sign-fixed sqrt branch (rodrigues.py:347-364)."""
    from pcd_reg_hregnet_amd.perturb import SE3
    L = SE3.log(cu(g["pi_g"])).cpu().numpy()
    np.testing.assert_allclose(L, g["pi_log"], atol=1e-5, rtol=0)


@pytest.mark.parametrize("tag,dist,randomly,seed", [("uniform_rand", "uniform", True, 3),
                                                    ("uniform_fixed", "uniform", False, 4),
                                                    ("gaussian_rand", "gaussian", True, 5),
                                                    ("invgauss_rand", "inverse_gaussian", True, 6)])
def test_uniform_transform_draws(g, tag, dist, randomly, seed):
    """Same seeds -> the reference's twists (the draws stay on torch's / numpy's CPU
    generators in the reference's order); the batch equals consecutive single draws."""
    from pcd_reg_hregnet_amd.perturb import UniformTransformSE3
    torch.manual_seed(seed)
    np.random.seed(seed)
    T = UniformTransformSE3(max_deg=20, max_tran=0.5, distribution=dist, mag_randomly=randomly)
    x = T.generate_transforms(24).cpu().numpy()
    np.testing.assert_allclose(x, g[f"twists_{tag}"], atol=2e-6, rtol=0)
    torch.manual_seed(seed)
    np.random.seed(seed)
    one = torch.cat([T.generate_transform() for _ in range(24)]).cpu().numpy()
    np.testing.assert_array_equal(one, x)


def test_apply_transform(g):
    from pcd_reg_hregnet_amd.perturb import UniformTransformSE3
    T = UniformTransformSE3(max_deg=20, max_tran=0.5, mag_randomly=True)
    out = T.apply_transform(cu(g["apply_p0"]), cu(g["apply_x"])).cpu().numpy()
    np.testing.assert_allclose(out, g["apply_out"], atol=2e-5, rtol=1e-6)
    np.testing.assert_allclose(T.gt.cpu().numpy(), g["apply_gt"], atol=1e-6, rtol=0)
    np.testing.assert_allclose(T.igt.cpu().numpy(), g["apply_igt"], atol=1e-6, rtol=0)


def test_lidar_to_lidar_from_file(g, tmp_path):
    """Validation split: twists from the perturbation file (man_dataset.py:500-507,
    617-625) -> uncalibed clouds, igt and the training loop's inverse(igt)."""
    from pcd_reg_hregnet_amd.perturb import PerturbationPipeline
    prefix = str(tmp_path / "perturbations_file_")
    np.savetxt(prefix + "val.txt", g["l2l_x"].astype(np.float64), delimiter=",")
    pipe = PerturbationPipeline(split="val", perturbations_file=prefix)
    r = pipe.lidar_to_lidar(cu(g["l2l_pcd"]), indices=[0, 1, 2, 3])
    np.testing.assert_allclose(r["uncalibed_pcd"].cpu().numpy(), g["l2l_uncalibed"], atol=2e-5,
                               rtol=1e-6)
    np.testing.assert_allclose(r["igt"].cpu().numpy(), g["l2l_igt"], atol=1e-6, rtol=0)
    np.testing.assert_allclose(r["gt"].cpu().numpy(), g["l2l_gt"], atol=2e-6, rtol=0)
    # permuted indices pick the matching twists
    r2 = pipe.lidar_to_lidar(cu(g["l2l_pcd"][::-1]), indices=[3, 2, 1, 0])
    assert torch.equal(r2["igt"], r["igt"].flip(0))


def test_train_split_matches_generator(g):
    """Train split: fresh twists per cloud, the same draws as UniformTransformSE3."""
    from pcd_reg_hregnet_amd.perturb import PerturbationPipeline, SE3, UniformTransformSE3
    pipe = PerturbationPipeline(split="train")
    torch.manual_seed(3)
    r = pipe.lidar_to_lidar(cu(g["l2l_pcd"]))
    np.testing.assert_allclose(r["twist"].cpu().numpy(), g["twists_uniform_rand"][:4], atol=2e-6,
                               rtol=0)
    assert torch.equal(r["igt"], SE3.exp(r["twist"]))
    eye = torch.eye(4, device="cuda").expand(4, 4, 4)
    torch.testing.assert_close(r["gt"] @ r["igt"], eye, atol=2e-6, rtol=0)


def test_create_perturb_file(g, tmp_path):
    """The perturbation file the reference writes for seed 7 (man_dataset.py:528-545)."""
    from pcd_reg_hregnet_amd.perturb import UniformTransformSE3, create_perturb_file, \
        load_perturb_file
    path = str(tmp_path / "p.txt")
    torch.manual_seed(7)
    create_perturb_file(path, 10, UniformTransformSE3(20, 0.5, "uniform", True))
    ref_path = tmp_path / "ref.txt"
    ref_path.write_text(str(g["perturb_file_text"]))
    ours, ref = load_perturb_file(path), load_perturb_file(str(ref_path))
    assert ours.shape == ref.shape == (10, 6)
    np.testing.assert_allclose(ours, ref, atol=2e-6, rtol=0)
    line = open(path).readline().strip().split(",")
    assert len(line) == 6 and all("e" in v for v in line)  # np.savetxt's %.18e


def test_range_filter_exact(g):
    from pcd_reg_hregnet_amd.perturb import PointCloudFilter
    f = PointCloudFilter(max_range=80)
    p, i, c = f.remove_points_by_range(cu(g["filter_in"]), cu(g["filter_in_int"]))
    np.testing.assert_array_equal(p.cpu().numpy(), g["filter_out"])
    np.testing.assert_array_equal(i.cpu().numpy(), g["filter_out_int"])
    # batched: every cloud packed independently, in order; an all-out cloud -> 0
    pts = g["filter_in"][:4096]
    batch = np.stack([pts, pts[::-1] * 1.5, pts * 100.0]).astype(np.float32)
    P, I, C = f.remove_points_by_range(cu(batch))
    for b in range(3):
        n = int(C[b])
        keep = np.sqrt((batch[b, :, 0] * batch[b, :, 0] + batch[b, :, 1] * batch[b, :, 1])
                       + batch[b, :, 2] * batch[b, :, 2]) < 80
        assert n == keep.sum()
        np.testing.assert_array_equal(P[b, :n].cpu().numpy(), batch[b][keep])
    assert int(C[2]) == 0
    e, _, ce = f.remove_points_by_range(torch.zeros(2, 0, 3, device="cuda"))
    assert ce.tolist() == [0, 0]


@pytest.mark.parametrize("tag", ["pad", "sub"])
def test_resampler_exact(g, tag):
    from pcd_reg_hregnet_amd.perturb import PointCloudResampler
    n = int(g[f"resample_{tag}_n"])
    np.random.seed(int(g[f"resample_{tag}_seed"]))
    rp, ri = PointCloudResampler(4096)(cu(g["filter_out"][:n]), cu(g["filter_out_int"][:n]))
    np.testing.assert_array_equal(rp.cpu().numpy(), g[f"resample_{tag}_out"])
    np.testing.assert_array_equal(ri.cpu().numpy(), g[f"resample_{tag}_int"])


def test_cpu_tensors_raise():
    from pcd_reg_hregnet_amd.perturb import SE3
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        SE3.exp(torch.zeros(2, 6))


def test_pipeline_feeds_the_forward_and_loss():
    """The reference's training-step data flow (train_reg_v0.py:263-294): perturb the
    calibrated dst cloud -> src = uncalibed, gt = inverse(igt) -> forward -> loss
    (the heads are seeded, not trained: only the plumbing is checked)."""
    from helpers import Args, state_dict_torch
    from pcd_reg_hregnet_amd import engine, losses, synthetic
    from pcd_reg_hregnet_amd.models import HRegNet
    from pcd_reg_hregnet_amd.perturb import PerturbationPipeline
    net = HRegNet(Args())
    net.load_state_dict(state_dict_torch())
    net = net.cuda().eval()
    _, d, _, _ = synthetic.lidar_batch(2, 4096, seed0=70)
    torch.manual_seed(0)
    r = PerturbationPipeline(split="train").lidar_to_lidar(cu(d))
    gt_R, gt_t = r["gt"][:, :3, :3].contiguous(), r["gt"][:, :3, 3].contiguous()
    with torch.no_grad():
        out = engine.hregnet_forward(net.prepared(torch.device("cuda")), r["uncalibed_pcd"], cu(d))
        l_trans, l_R, l_t = losses.transformation_loss(out["rotation"][-1], out["translation"][-1],
                                                       gt_R, gt_t, 1.0)[:3]
    assert torch.isfinite(l_trans) and float(l_R) >= 0 and float(l_t) >= 0
    # gt maps the uncalibed cloud back onto the calibrated one
    back = torch.einsum("bij,bnj->bni", gt_R, r["uncalibed_pcd"]) + gt_t[:, None]
    torch.testing.assert_close(back, cu(d), atol=2e-4, rtol=0)
