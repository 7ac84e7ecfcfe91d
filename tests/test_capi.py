"""The C-ABI library: every symbol include/hregnet_amd.h declares is exported, and the
ctypes signatures in pcd_reg_hregnet_amd/_lib.py agree with the header (no GPU needed); the
same for the test-only checker library (include/hregnet_amd_checkers.h ->
libhregnet_checkers.so), whose symbols the product library must NOT carry."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "hregnet_amd.h")
CHECKER_HEADER = os.path.join(REPO, "include", "hregnet_amd_checkers.h")


def _declared(header=HEADER):
    text = open(header).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    decls = {}
    for m in re.finditer(r"(?:int|size_t|const char \*)\s*(hreg_\w+)\s*\(([^;]*?)\)\s*;", text, flags=re.S):
        params = [p.strip() for p in m.group(2).split(",") if p.strip() and p.strip() != "void"]
        decls[m.group(1)] = len(params)
    return decls


@pytest.fixture(scope="module")
def lib():
    from pcd_reg_hregnet_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        from pcd_reg_hregnet_amd import build
        build.build()
    return _lib


def test_header_parses():
    d = _declared()
    for name in ("hreg_furthest_point_sampling", "hreg_weighted_furthest_point_sampling",
                 "hreg_gather_points", "hreg_gather_points_grad", "hreg_knn_points",
                 "hreg_knn_gather", "hreg_gemm", "hreg_weighted_svd"):
        assert name in d


def test_library_exports_every_declared_symbol(lib):
    L = ctypes.CDLL(lib.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(L, n)]
    assert not missing, missing


def test_ctypes_signatures_match_header(lib):
    d = _declared()
    for name, args in lib._SIGS.items():
        assert name in d, f"{name} bound in _lib but not declared in the header"
        assert len(args) == d[name], (name, len(args), d[name])
    for name in d:
        assert name in lib.EXPORTS, f"{name} declared but not bound in _lib"


def test_checker_library_is_separate(lib):
    """the fp32-MFMA twin kernels live only in the checker library, bound with the header's
    arity; the product library exports none of them"""
    d = _declared(CHECKER_HEADER)
    assert set(d) == set(lib.CHECKER_EXPORTS), (sorted(d), lib.CHECKER_EXPORTS)
    for name, args in lib._CHECKER_SIGS.items():
        assert len(args) == d[name], name
    C = ctypes.CDLL(lib.CHECKER_PATH)
    P = ctypes.CDLL(lib.LIB_PATH)
    for name in d:
        assert hasattr(C, name), name
        assert not hasattr(P, name), f"{name} is in the product library"


def test_load_without_gpu_is_allowed_but_ops_fail_loudly(lib):
    import torch
    L = lib.load(require_gpu=False)
    assert L.hreg_version().startswith(b"hregnet_amd")
    if not torch.cuda.is_available():
        with pytest.raises(RuntimeError, match="no GPU"):
            lib.load()


def test_struct_layout_matches_c():
    """hreg_seg_t / hreg_gemm_t sizes as the C compiler lays them out."""
    import subprocess
    import tempfile
    from pcd_reg_hregnet_amd import _lib
    src = ('#include "hregnet_amd.h"\n#include <stdio.h>\n#include <stddef.h>\n'
           'int main(){printf("%zu %zu %zu %zu\\n", sizeof(hreg_seg_t), sizeof(hreg_gemm_t),'
           ' offsetof(hreg_gemm_t, W), offsetof(hreg_gemm_t, out_batch_stride));return 0;}')
    with tempfile.TemporaryDirectory() as td:
        c = os.path.join(td, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(td, "t")
        subprocess.check_call(["gcc", "-I", os.path.join(REPO, "include"), c, "-o", exe])
        sizes = [int(v) for v in subprocess.check_output([exe]).split()]
    assert sizes == [ctypes.sizeof(_lib.Seg), ctypes.sizeof(_lib.Gemm),
                     _lib.Gemm.W.offset, _lib.Gemm.out_batch_stride.offset]
