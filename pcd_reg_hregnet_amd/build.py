"""Build the gfx950 HIP library ``libhregnet_amd.so`` in-tree with hipcc.

Used by ``__graft_entry__.build()`` and ``python -m pcd_reg_hregnet_amd.build``.
Each ``csrc/*.hip`` is compiled to an object (in parallel), then linked into
one shared library next to this file, so it travels to the GPU box with the
repo snapshot.  ``csrc/checkers/*.hip`` (the fp32-MFMA twins of the level kernels,
test checkers only) go into a separate ``libhregnet_checkers.so`` that the product path
never loads (include/hregnet_amd_checkers.h).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJDIR = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "libhregnet_amd.so")
CHECKERS = os.path.join(CSRC, "checkers")
CHECKER_LIB = os.path.join(HERE, "libhregnet_checkers.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("HREG_ARCH", "gfx950")

CFLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off",
    "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
]


# Kernels running v_mfma_f32_32x32x16_bf16 (the bf16x6 split products) are compiled
# without packed fp32 VALU ops (v_pk_mul_f32 / v_pk_add_f32): with them, group_l1_6 gave
# nondeterministic wrong accumulator values whenever two waves shared a SIMD (two
# workgroups per CU, or one 8-wave workgroup), and exact results with one wave per SIMD
# or without the packed ops (tools/debug_l1_6.py; the instruction
# pairings suspected so far are ruled out by tools/micro/pk_hazard.hip).  The flag is
# derived, not listed: every source that uses the bf16x6 headers or names the bf16 MFMA
# gets it, and tests/test_isa.py fails if any built kernel still mixes the two.  The
# host-side compile ignores the feature (a warning).
NO_PACKED_F32 = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
B6_MARKERS = ("mfma_chain.h", "split_chain.h", "mfma_jt.h", "mfma_f32_32x32x16_bf16")


def uses_bf16_mfma(path: str) -> bool:
    with open(path) as f:
        text = f.read()
    return any(m in text for m in B6_MARKERS)


def file_flags(path: str) -> list[str]:
    return NO_PACKED_F32 if uses_bf16_mfma(path) else []


def _needs(obj: str, deps: list[str]) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src: str, obj: str, extra=()) -> tuple[str, int, str]:
    cmd = [HIPCC, *CFLAGS, *file_flags(src), *extra, "-c", src, "-o", obj]
    p = subprocess.run(cmd, capture_output=True, text=True)
    return src, p.returncode, p.stdout + p.stderr


def _build_lib(srcs, objdir, lib, headers, verbose, force, extra=()) -> str:
    os.makedirs(objdir, exist_ok=True)
    jobs = []
    objs = []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s).replace(".hip", ".o"))
        objs.append(o)
        if force or _needs(o, [s, *headers]):
            jobs.append((s, o))
    if jobs:
        with cf.ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
            for src, rc, log in ex.map(lambda a: _compile(*a, extra), jobs):
                if verbose or rc:
                    sys.stderr.write(f"[hipcc] {os.path.basename(src)} rc={rc}\n{log}")
                if rc:
                    raise RuntimeError(f"hipcc failed for {src}")
    if force or jobs or _needs(lib, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib, *objs]
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode:
            raise RuntimeError("link failed:\n" + p.stdout + p.stderr)
    return lib


def build(verbose: bool = False, force: bool = False) -> str:
    headers = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(
        os.path.join(HERE, "..", "include", "*.h")) + [os.path.abspath(__file__)]
    _build_lib(sorted(glob.glob(os.path.join(CHECKERS, "*.hip"))), os.path.join(OBJDIR, "checkers"),
               CHECKER_LIB, headers, verbose, force)
    return _build_lib(sorted(glob.glob(os.path.join(CSRC, "*.hip"))), OBJDIR, LIB, headers, verbose,
                      force)


def variant(name: str, defines: list[str], verbose: bool = False) -> str:
    """A/B build of the core library with extra -D switches (the csrc/*.hip HREG_* compile
    switches) into pcd_reg_hregnet_amd/ab_<name>.so, loaded by HREG_LIB (tools/gpu_abn.sh
    lib:ab_<name>.so).  Always a full rebuild: a variant must export what the tree does."""
    headers = []
    return _build_lib(sorted(glob.glob(os.path.join(CSRC, "*.hip"))), os.path.join(OBJDIR, "ab_" + name),
                      os.path.join(HERE, f"ab_{name}.so"), headers, verbose, True,
                      [f"-D{d}" for d in defines])


if __name__ == "__main__":
    # python -m pcd_reg_hregnet_amd.build [-v] [-f] | --variant NAME DEF=V ...
    if "--variant" in sys.argv:
        i = sys.argv.index("--variant")
        print(variant(sys.argv[i + 1], sys.argv[i + 2:], verbose="-v" in sys.argv[:i]))
    else:
        print(build(verbose="-v" in sys.argv, force="-f" in sys.argv))
