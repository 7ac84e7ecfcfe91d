"""Build the gfx950 HIP library ``libhregnet_amd.so`` in-tree with hipcc.

Used by ``__graft_entry__.build()`` and ``python -m pcd_reg_hregnet_amd.build``.
Each ``csrc/*.hip`` is compiled to an object (in parallel), then linked into
one shared library next to this file, so it travels to the GPU box with the
repo snapshot.
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
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("HREG_ARCH", "gfx950")

CFLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off",
    "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
]


def _needs(obj: str, deps: list[str]) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src: str, obj: str) -> tuple[str, int, str]:
    cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
    p = subprocess.run(cmd, capture_output=True, text=True)
    return src, p.returncode, p.stdout + p.stderr


def build(verbose: bool = False, force: bool = False) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    headers = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(
        os.path.join(HERE, "..", "include", "*.h"))
    jobs = []
    objs = []
    for s in srcs:
        o = os.path.join(OBJDIR, os.path.basename(s).replace(".hip", ".o"))
        objs.append(o)
        if force or _needs(o, [s, *headers]):
            jobs.append((s, o))
    if jobs:
        with cf.ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
            for src, rc, log in ex.map(lambda a: _compile(*a), jobs):
                if verbose or rc:
                    sys.stderr.write(f"[hipcc] {os.path.basename(src)} rc={rc}\n{log}")
                if rc:
                    raise RuntimeError(f"hipcc failed for {src}")
    if force or jobs or _needs(LIB, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode:
            raise RuntimeError("link failed:\n" + p.stdout + p.stderr)
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv, force="-f" in sys.argv))
