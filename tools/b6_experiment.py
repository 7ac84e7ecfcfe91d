"""Where the time of the bf16x6 level kernels goes: variants with parts removed
(mfma_chain.h HREG_B6_EXP; results are wrong, only the timing means anything), timed
on random inputs at config-2 sizes (16 clouds).

  0: the product kernels; 2: no weight-piece loads; 5: B not split into pieces.
usage: python tools/b6_experiment.py build   (here: builds tools/b6exp_<v>.so)
       python tools/b6_experiment.py [v ...] (GPU box: times the built variants, all by default)"""
import ctypes
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
VARIANTS = (0, 2, 5)
SRCS = ("group_l1_6.hip", "group_fused6.hip", "group_split6.hip", "coarse6.hip")


def so_path(v):
    return os.path.join(REPO, "tools", f"b6exp_{v}.so")


def build():
    from pcd_reg_hregnet_amd import build as b
    for v in VARIANTS:
        objs = []
        for src in SRCS:
            obj = f"/tmp/b6exp_{v}_{src}.o"
            extra = os.environ.get("B6EXP_DEFS", "").split()  # e.g. -DHREG_L1_LDSW=1
            subprocess.check_call([b.HIPCC, *b.CFLAGS, *b.FILE_FLAGS.get(src, []), f"-DHREG_B6_EXP={v}", *extra, "-c",
                                   os.path.join(b.CSRC, src), "-o", obj])
            objs.append(obj)
        subprocess.check_call([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", so_path(v), *objs])
        print(so_path(v))


def run():
    import torch
    from tools.op_bench import timeit
    torch.cuda.init()
    rng = np.random.default_rng(0)
    vp = ctypes.c_void_p
    st = torch.cuda.current_stream().cuda_stream

    def t(x):
        return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).cuda()

    res = {}
    for v in [int(a) for a in sys.argv[1:]] or VARIANTS:
        if not os.path.exists(so_path(v)):
            continue
        L = ctypes.CDLL(so_path(v))
        for name in ("hreg_group_l1_6", "hreg_group6_l2", "hreg_group_split6_l3", "hreg_coarse_head6",
                     "hreg_group6x2_l2"):
            if hasattr(L, name + "_table_floats"):
                getattr(L, name + "_table_floats").restype = ctypes.c_int
            getattr(L, name).restype = ctypes.c_int
        # level 1: 16 x 1024 groups of 64 rows
        G = 16 * 1024
        tb = t(rng.normal(0, 0.05, L.hreg_group_l1_6_table_floats()))
        geom, kx = t(rng.normal(size=(G * 64, 4))), t(rng.normal(size=(G * 64, 3)))
        kp, att, desc = torch.empty(G, 3, device="cuda"), torch.empty(G, 64, device="cuda"), \
            torch.empty(G, 64, device="cuda")
        f1 = lambda: L.hreg_group_l1_6(vp(tb.data_ptr()), vp(geom.data_ptr()), vp(kx.data_ptr()), G,  # noqa: E731
                                       vp(kp.data_ptr()), vp(att.data_ptr()), vp(desc.data_ptr()), vp(st))
        res[f"l1_{v}_us"] = round(timeit(f1, reps=20) * 1e3, 1)
        # levels 2 / 3 (pre path): G groups of KN rows gathering nrows source points
        for name, G, KN, CF, T1, C3, CM2, nrows in (("hreg_group6_l2", 16 * 512, 32, 64, 2, 128, 128, 16 * 1024),
                                                    ("hreg_group6x2_l2", 16 * 512, 32, 64, 2, 128, 128, 16 * 1024),
                                                    ("hreg_group_split6_l3", 16 * 256, 16, 128, 4, 256, 256,
                                                     16 * 512)):
            tb = t(rng.normal(0, 0.05, getattr(L, name.replace("6x2", "6") + "_table_floats")()))
            geom, kx = t(rng.normal(size=(G * KN, 4))), t(rng.normal(size=(G * KN, 3)))
            gidx = torch.from_numpy(rng.integers(0, nrows, G * KN).astype(np.int32)).cuda()
            feats = t(np.abs(rng.normal(size=(nrows, CF))))
            pre = t(rng.normal(size=(nrows, 2 * T1 * 32)))
            kp, att, desc = torch.empty(G, 3, device="cuda"), torch.empty(G, C3, device="cuda"), \
                torch.empty(G, CM2, device="cuda")
            fn = getattr(L, name)
            f = lambda: fn(vp(tb.data_ptr()), vp(geom.data_ptr()), vp(kx.data_ptr()), vp(gidx.data_ptr()),  # noqa: E731
                           vp(feats.data_ptr()), G, vp(kp.data_ptr()), vp(att.data_ptr()), vp(desc.data_ptr()),
                           vp(pre.data_ptr()), vp(st))
            res[f"{name}_{v}_us"] = round(timeit(f, reps=20) * 1e3, 1)
        # CoarseReg convs_1 + attention: 8 pairs x 256 keypoints, 8 neighbours, 256 destinations
        G, N = 8 * 256, 8 * 256
        tb = t(rng.normal(0, 0.03, L.hreg_coarse_head6_table_floats()))
        small = t(rng.normal(size=(G * 8, 16)))
        ud0, ud1 = t(rng.normal(size=(G, 512))), t(rng.normal(size=(N, 512)))
        gidx = torch.from_numpy(rng.integers(0, N, G * 8).astype(np.int32)).cuda()
        kx = t(rng.normal(size=(G * 8, 3)))
        corres, att = torch.empty(G, 3, device="cuda"), torch.empty(G, 512, device="cuda")
        fc = lambda: L.hreg_coarse_head6(vp(tb.data_ptr()), vp(small.data_ptr()), vp(ud0.data_ptr()),  # noqa: E731
                                         vp(ud1.data_ptr()), vp(gidx.data_ptr()), vp(kx.data_ptr()), G,
                                         vp(corres.data_ptr()), vp(att.data_ptr()), vp(st))
        res[f"coarse6_{v}_us"] = round(timeit(fc, reps=20) * 1e3, 1)
        print(v, {k: x for k, x in res.items() if k.endswith(f"_{v}_us")}, flush=True)
    print(res)


if __name__ == "__main__":
    build() if sys.argv[1:] == ["build"] else run()
