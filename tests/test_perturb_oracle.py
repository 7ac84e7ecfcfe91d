"""CPU: the oracle's restatement of the data side (oracle.se3_exp / se3_log /
twists_from_samples / range_filter / resample_indices) against the fixtures the
reference produced (tests/golden/perturb.npz), and the host-side draw order of
pcd_reg_hregnet_amd.perturb (no GPU call)."""
import math

import numpy as np
import pytest
import torch

from helpers import load_npz
from oracle import oracle as O


@pytest.fixture(scope="module")
def g():
    return load_npz("perturb.npz")


def test_oracle_se3(g):
    ang = np.linalg.norm(g["se3_x"][:, :3], axis=1)
    np.testing.assert_allclose(O.se3_exp(g["se3_x"]), g["se3_exp"], atol=1e-6, rtol=0)
    L = O.se3_log(g["se3_exp"])
    np.testing.assert_allclose(L[ang < 3.0], g["se3_log"][ang < 3.0], atol=1e-5, rtol=0)
    np.testing.assert_allclose(L[ang >= 3.0], g["se3_log"][ang >= 3.0], atol=5e-4, rtol=0)
    np.testing.assert_allclose(O.se3_log(g["pi_g"]), g["pi_log"], atol=1e-6, rtol=0)


@pytest.mark.parametrize("tag,dist,randomly,seed", [("uniform_rand", "uniform", True, 3),
                                                    ("uniform_fixed", "uniform", False, 4),
                                                    ("gaussian_rand", "gaussian", True, 5),
                                                    ("invgauss_rand", "inverse_gaussian", True, 6)])
def test_oracle_twists_and_draw_order(g, tag, dist, randomly, seed):
    from pcd_reg_hregnet_amd.perturb import _draws
    torch.manual_seed(seed)
    np.random.seed(seed)
    mags, s = _draws(24, randomly, dist)
    at = np.array([((m[0] * 20 if randomly else 20) * math.pi / 180.0,
                    (m[1] * 0.5 if randomly else 0.5)) for m in mags], np.float32)
    np.testing.assert_allclose(O.twists_from_samples(s, at, dist), g[f"twists_{tag}"], atol=2e-7,
                               rtol=0)


def test_oracle_filter_and_resampler(g):
    p, i = O.range_filter(g["filter_in"], g["filter_in_int"], 80)
    np.testing.assert_array_equal(p, g["filter_out"])
    np.testing.assert_array_equal(i, g["filter_out_int"])
    for tag in ("pad", "sub"):
        n = int(g[f"resample_{tag}_n"])
        np.random.seed(int(g[f"resample_{tag}_seed"]))
        idx = O.resample_indices(n, 4096)
        np.testing.assert_array_equal(g["filter_out"][:n][idx], g[f"resample_{tag}_out"])
        np.testing.assert_array_equal(g["filter_out_int"][:n][idx], g[f"resample_{tag}_int"])
