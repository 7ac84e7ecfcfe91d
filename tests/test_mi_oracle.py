"""CPU: the oracle's restatement of Model_V2's training losses (oracle.deep_mi_loss,
oracle.chamfer_loss) against the reference's own losses/mi_loss_v2.py and
losses/chamfer_loss.py outputs (tests/golden/mi_chamfer.npz)."""
import numpy as np
import pytest

from helpers import load_npz
from oracle import oracle as O


@pytest.fixture(scope="module")
def g():
    return load_npz("mi_chamfer.npz")


def test_oracle_deep_mi(g):
    params = {k[6:]: g[k] for k in g if k.startswith("param_")}
    args = [g["in_" + k] for k in ("x_global", "x_global_prime", "x_local", "x_local_prime",
                                    "c_local", "c_global")]
    tot, loc, glo = O.deep_mi_loss(params, *args)
    np.testing.assert_allclose([tot, loc, glo], [g["loss"], g["loss_local"], g["loss_global"]],
                               rtol=1e-6)


@pytest.mark.parametrize("red", ["mean", "none", "sum"])
def test_oracle_chamfer(g, red):
    np.testing.assert_allclose(O.chamfer_loss(g["chamfer_a"], g["chamfer_b"], 50.0, red),
                               g["chamfer_" + red], rtol=1e-6)
