"""Build an alternative libhregnet_amd (A/B and hazard experiments): csrc files
(comma-separated) recompiled with extra -D flags, linked with the other in-tree objects.
usage: python tools/build_variant.py OUT.so csrc_file.hip[,other.hip] -DNAME=VALUE ... [--packed]
(--packed: without build.NO_PACKED_F32, the packed-fp32 hazard reproduction)
Select it at run time with HREG_LIB=OUT.so."""
import glob, os, subprocess, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pcd_reg_hregnet_amd import build as b

out, srcs, defs = sys.argv[1], sys.argv[2].split(","), sys.argv[3:]
b.build()
new = []
for src in srcs:
    obj = out + "." + src.replace(".hip", ".o")
    flags = [] if "--packed" in defs else b.file_flags(os.path.join(b.CSRC, src))
    subprocess.check_call([b.HIPCC, *b.CFLAGS, *flags, *[d for d in defs if d != "--packed"], "-c",
                           os.path.join(b.CSRC, src), "-o", obj])
    new.append(obj)
skip = {s.replace(".hip", ".o") for s in srcs}
objs = [o for o in sorted(glob.glob(os.path.join(b.OBJDIR, "*.o"))) if os.path.basename(o) not in skip] + new
subprocess.check_call([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", out, *objs])
for obj in new:
    os.remove(obj)
print(out)
