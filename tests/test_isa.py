"""ISA checks on the built gfx950 code objects (no GPU needed): no kernel that issues the
bf16 MFMA of the bf16x6 products also issues packed-fp32 VALU ops (the
nondeterministic-accumulator defect of DESIGN.md 4b appeared with exactly that mix), and
the build derives that flag for every source that needs it."""
import glob
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
PACKED = re.compile(r"\bv_pk_(add|mul|fma|mov)_(f32|b32)\b")


def _disasm(obj, tmp):
    fat, elf = os.path.join(tmp, "fat.bin"), os.path.join(tmp, "dev.elf")
    subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj])
    subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={elf}"])
    return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", elf], check=True,
                          capture_output=True, text=True).stdout


def _kernels(text):
    """function name -> its instruction lines"""
    out, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            out[cur] = []
        elif cur is not None and line.startswith("\t"):
            out[cur].append(line)
    return out


@pytest.fixture(scope="module")
def objects():
    from pcd_reg_hregnet_amd import build
    if not os.path.isdir(os.path.join(build.OBJDIR)) or not os.path.exists(build.LIB):
        build.build()
    objs = sorted(glob.glob(os.path.join(build.OBJDIR, "*.o")))
    assert objs
    return objs


def test_no_packed_fp32_beside_bf16_mfma(objects, tmp_path):
    checked = 0
    for obj in objects:
        for name, lines in _kernels(_disasm(obj, str(tmp_path))).items():
            if not any("v_mfma_f32_32x32x16_bf16" in ln for ln in lines):
                continue
            checked += 1
            bad = [ln.strip() for ln in lines if PACKED.search(ln)]
            assert not bad, (os.path.basename(obj), name, bad[:3])
    assert checked >= 10  # the bf16x6 kernel family is present


def test_flag_derived_for_every_bf16x6_source():
    from pcd_reg_hregnet_amd import build
    srcs = glob.glob(os.path.join(build.CSRC, "*.hip"))
    need = {os.path.basename(s) for s in srcs if build.uses_bf16_mfma(s)}
    for s in ("group_l1_6.hip", "group_fused6.hip", "group_split6.hip", "group_head.hip",
              "coarse6.hip", "mlp_head.hip", "gemm.hip"):
        assert s in need
    for s in srcs:
        assert (build.file_flags(s) == build.NO_PACKED_F32) == (os.path.basename(s) in need)
