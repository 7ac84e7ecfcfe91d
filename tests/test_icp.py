"""Point-to-point ICP refinement (reference test/test_v4.py:140-158, open3d
registration_icp; open3d is not vendored, so its published loop is restated in
oracle/oracle.py registration_icp and the GPU path, csrc/icp.hip, is held to that
restatement; parity unpinned against open3d itself)."""
import numpy as np
import pytest
import torch

from oracle import oracle


def _rot(rng, deg):
    from scipy.spatial.transform import Rotation
    return Rotation.from_rotvec(np.deg2rad(deg) * rng.normal(size=3) / np.sqrt(3)).as_matrix()


def _planted(rng, n=3000, deg=4.0, tr=0.3):
    """target cloud, source = T^-1 applied to a noiseless subset: ICP from identity must
    find T (source -> target)"""
    dst = rng.uniform(-20, 20, (n, 3)).astype(np.float32)
    R = _rot(rng, deg)
    t = rng.uniform(-tr, tr, 3)
    src = ((dst[: n // 2].astype(np.float64) - t) @ R).astype(np.float32)  # R^T (x - t)
    T = np.eye(4)
    T[:3, :3], T[:3, 3] = R, t
    return src, dst, T


def test_oracle_icp_recovers_planted_transform():
    rng = np.random.default_rng(0)
    src, dst, T = _planted(rng)
    Tf, fit, rmse, it = oracle.registration_icp(src, dst, 1.0, max_iteration=100)
    assert fit == 1.0 and rmse < 1e-5 and 1 <= it < 100
    np.testing.assert_allclose(Tf, T, atol=1e-5)


def test_oracle_icp_zero_iterations_and_no_matches():
    rng = np.random.default_rng(1)
    src, dst, _ = _planted(rng, n=400)
    T0 = np.eye(4)
    T0[:3, 3] = 500.0  # far away: no correspondence within 1 m
    Tf, fit, rmse, it = oracle.registration_icp(src, dst, 1.0, init=T0, max_iteration=10)
    assert fit == 0.0 and rmse == 0.0 and it == 1  # identity update, then converged
    np.testing.assert_array_equal(Tf, T0)
    Tf, fit, _, it = oracle.registration_icp(src, dst, 1.0, max_iteration=0)
    assert it == 0 and np.array_equal(Tf, np.eye(4))


def _gpu_icp(src, dst, init, max_iter, r=1.0):
    from pcd_reg_hregnet_amd import icp
    res = icp.registration_icp(torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda(), r,
                               init=None if init is None else torch.from_numpy(init.astype(np.float32)).cuda(),
                               criteria=icp.ICPConvergenceCriteria(1e-6, 1e-6, max_iter))
    torch.cuda.synchronize()
    return (res.transformation.cpu().numpy(), res.fitness.cpu().numpy(),
            res.inlier_rmse.cpu().numpy(), res.iterations.cpu().numpy())


@pytest.mark.gpu
def test_gpu_icp_recovers_planted_transform():
    rng = np.random.default_rng(0)
    src, dst, T = _planted(rng)
    Tf, fit, rmse, it = _gpu_icp(src, dst, None, 100)
    assert fit == 1.0 and rmse < 1e-5 and 1 <= it < 100
    np.testing.assert_allclose(Tf, T, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [4096, 16384])
def test_gpu_icp_matches_oracle_on_lidar_pairs(n):
    """A batch of KITTI-shape pairs from a perturbed ground-truth start: every pair's final
    pose, fitness, rmse and iteration count against the oracle restatement."""
    from pcd_reg_hregnet_amd import synthetic
    B = 3
    s, d, Rg, tg = synthetic.lidar_batch(B, n, seed0=70)
    rng = np.random.default_rng(2)
    inits = []
    for b in range(B):
        # a start near the pose that maps src onto dst, dst = R_gt src + t_gt (the network's
        # output plays this role in test_v4)
        T0 = np.eye(4)
        T0[:3, :3] = _rot(rng, 3.0) @ Rg[b].astype(np.float64)
        T0[:3, 3] = tg[b] + rng.uniform(-0.3, 0.3, 3)
        inits.append(T0)
    inits = np.stack(inits)
    from pcd_reg_hregnet_amd import icp
    res = icp.registration_icp(torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda(), 1.0,
                               init=torch.from_numpy(inits.astype(np.float32)).cuda(),
                               criteria=icp.ICPConvergenceCriteria(1e-6, 1e-6, 60))
    torch.cuda.synchronize()
    for b in range(B):
        T, fit, rmse, it = oracle.registration_icp(s[b], d[b], 1.0,
                                                   init=inits[b].astype(np.float32).astype(np.float64),
                                                   max_iteration=60)
        print(f"pair {b}: updates gpu {int(res.iterations[b])} oracle {it}, fitness "
              f"{float(res.fitness[b]):.6f} / {fit:.6f}, rmse {float(res.inlier_rmse[b]):.6f} / {rmse:.6f}")
        assert int(res.iterations[b]) == it
        assert abs(float(res.fitness[b]) - fit) <= 1e-6
        assert abs(float(res.inlier_rmse[b]) - rmse) <= 1e-5 * max(rmse, 1.0)
        np.testing.assert_allclose(res.transformation[b].cpu().numpy(), T, atol=1e-5)
