"""Build an alternative libhregnet_amd (A/B and hazard experiments): one csrc file
recompiled with extra -D flags, linked with the other in-tree objects.
usage: python tools/build_variant.py OUT.so csrc_file.hip -DNAME=VALUE ...
Select it at run time with HREG_LIB=OUT.so."""
import glob, os, subprocess, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pcd_reg_hregnet_amd import build as b

out, src, defs = sys.argv[1], sys.argv[2], sys.argv[3:]
b.build()
srcp = os.path.join(b.CSRC, src)
obj = out + "." + src.replace(".hip", ".o")
subprocess.check_call([b.HIPCC, *b.CFLAGS, *b.FILE_FLAGS.get(src, []), *defs, "-c", srcp, "-o", obj])
objs = [o for o in sorted(glob.glob(os.path.join(b.OBJDIR, "*.o")))
        if os.path.basename(o) != src.replace(".hip", ".o")] + [obj]
subprocess.check_call([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", out, *objs])
os.remove(obj)
print(out)
