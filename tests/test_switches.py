"""The package's runtime switches stay few and measured: every
``switches.flag`` name the modules declare has a row in DESIGN.md section 12.4's table (the
measurement that keeps it), and there are at most 12 of them."""
import importlib
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODULES = ("engine", "train", "train_graph", "trainer", "models", "knn", "icp", "perturb", "losses",
           "mi_losses", "metrics", "utils", "point_utils_cuda")


def _declared():
    from pcd_reg_hregnet_amd import switches
    for m in MODULES:
        importlib.import_module(f"pcd_reg_hregnet_amd.{m}")
    return set(switches._USED)


def _table_rows():
    text = open(os.path.join(ROOT, "DESIGN.md")).read()
    sec = text[text.index("### 12.4 Switches"):]
    sec = sec[:sec.index("\n### ", 1)]
    return set(re.findall(r"^\| `([A-Z0-9_]+)` \|", sec, re.M))


def test_every_switch_has_its_measurement_row():
    missing = _declared() - _table_rows()
    assert not missing, f"switches without a DESIGN.md 12.4 row: {sorted(missing)}"


def test_switch_count_bounded():
    assert len(_declared()) <= 12
