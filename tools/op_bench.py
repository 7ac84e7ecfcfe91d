"""Micro-benchmarks of single C-ABI ops on the GPU (HIP events, median of reps).

usage: python tools/op_bench.py fps|fps64k|wfps|knn|l2|all [--b 16]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pcd_reg_hregnet_amd import _lib, engine  # noqa: E402


def timeit(fn, reps=10, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", default="all", nargs="?")
    ap.add_argument("--b", type=int, default=16)
    a = ap.parse_args()
    _lib.load()
    rng = np.random.default_rng(0)
    res = {}
    if a.what in ("fps", "all"):
        x = torch.from_numpy(rng.uniform(-40, 40, (a.b, 16384, 3)).astype(np.float32)).cuda()
        res["fps_l1_ms"] = timeit(lambda: engine.fps(x, 1024))
    if a.what in ("fps64k", "all"):
        # config 5 level 1: 2 pairs -> 4 clouds of 65536 points (multi-workgroup FPS)
        for nb in (4, 16):
            x = torch.from_numpy(rng.uniform(-40, 40, (nb, 65536, 3)).astype(np.float32)).cuda()
            res[f"fps_65536_b{nb}_ms"] = timeit(lambda: engine.fps(x, 1024))
        p = x[:4].contiguous()
        q = p[:, :1024].contiguous()
        res["knn_group_65536_b4_ms"] = timeit(lambda: engine.knn_group(q, p, 64))
    if a.what in ("wfps", "all"):
        for n, m in ((1024, 512), (512, 256)):
            x = torch.from_numpy(rng.uniform(-40, 40, (a.b, n, 3)).astype(np.float32)).cuda()
            w = torch.from_numpy(rng.uniform(0.5, 2, (a.b, n)).astype(np.float32)).cuda()
            res[f"wfps_{n}_ms"] = timeit(lambda: engine.fps(x, m, w))
    if a.what in ("knn", "all"):
        p = torch.from_numpy(rng.uniform(-40, 40, (a.b, 16384, 3)).astype(np.float32)).cuda()
        q = p[:, :1024].contiguous()
        res["knn_group_l1_ms"] = timeit(lambda: engine.knn_group(q, p, 64))
        ws = torch.empty(engine.spatial_index_bytes(a.b, 16384), dtype=torch.uint8, device="cuda")
        res["knn_group_l1_indexed_ms"] = timeit(lambda: engine.knn_group_indexed(q, p, 64, ws))
        res["spatial_index_ms"] = timeit(lambda: _lib.call("hreg_spatial_index", p, a.b, 16384, ws,
                                                           _lib.stream_handle()))
        from pcd_reg_hregnet_amd import synthetic
        pl = torch.from_numpy(synthetic.lidar_batch(a.b // 2, 16384, seed0=0)[1]).cuda()
        pl = torch.cat([pl, pl], 0).contiguous()
        ql = pl[:, ::16].contiguous()
        res["knn_group_l1_lidar_ms"] = timeit(lambda: engine.knn_group(ql, pl, 64))
        res["knn_group_l1_lidar_indexed_ms"] = timeit(lambda: engine.knn_group_indexed(ql, pl, 64, ws))
        d = torch.from_numpy(rng.normal(size=(a.b // 2, 256, 256)).astype(np.float32)).cuda()
        res["knn_desc_ms"] = timeit(lambda: engine.knn_idx32(d, d, 8))
    if a.what in ("l2", "all"):
        L = _lib.load()
        G = a.b * 512
        nt = L.hreg_group_l2_table_floats()
        tb = torch.from_numpy(rng.normal(0, 0.1, nt).astype(np.float32)).cuda()
        geom = torch.from_numpy(rng.normal(size=(G * 32, 4)).astype(np.float32)).cuda()
        kx = torch.from_numpy(rng.normal(size=(G * 32, 3)).astype(np.float32)).cuda()
        gidx = torch.from_numpy(rng.integers(0, a.b * 1024, G * 32).astype(np.int32)).cuda()
        feats = torch.from_numpy(rng.normal(size=(a.b * 1024, 64)).astype(np.float32)).cuda()
        kp = torch.empty(G, 3, device="cuda")
        att = torch.empty(G, 128, device="cuda")
        desc = torch.empty(G, 128, device="cuda")
        res["group_l2_ms"] = timeit(lambda: _lib.call("hreg_group_l2", tb, geom, kx, gidx, feats, G,
                                                      kp, att, desc, _lib.stream_handle()))
        flops = 2.0 * 32 * (2 * (68 * 64 + 64 * 64 + 64 * 128) + 384 * 64 + 64 * 128) * G
        res["group_l2_tflops"] = flops / res["group_l2_ms"] / 1e9
    if a.what in ("perturb", "all"):
        # data side (perturb.hip): L2L perturbation of 64 clouds x 16384 points (HBM:
        # 12 B in + 12 B out per point) and the range filter over 64 raw clouds of
        # 65536 points (12 B in + <= 12 B out per point)
        from pcd_reg_hregnet_amd import perturb
        B, N = 64, 16384
        pts = torch.from_numpy(rng.uniform(-60, 60, (B, N, 3)).astype(np.float32)).cuda()
        x = torch.from_numpy(rng.normal(0, 0.2, (B, 6)).astype(np.float32)).cuda()
        out = torch.empty_like(pts)
        igt = torch.empty(B, 16, device="cuda")
        gt = torch.empty(B, 16, device="cuda")
        ms = timeit(lambda: _lib.call("hreg_perturb_clouds", pts, x, B, N, out, igt, gt,
                                      _lib.stream_handle()), reps=20)
        res["perturb_clouds_64x16384_us"] = ms * 1e3
        res["perturb_clouds_GBps"] = B * N * 24 / ms / 1e6
        N2 = 65536
        raw = torch.from_numpy(rng.uniform(-100, 100, (B, N2, 3)).astype(np.float32)).cuda()
        filt = perturb.PointCloudFilter(80.0)
        ms = timeit(lambda: filt.remove_points_by_range(raw), reps=20)
        kept = int(filt.remove_points_by_range(raw)[2].sum())
        res["range_filter_64x65536_us"] = ms * 1e3
        res["range_filter_GBps"] = (B * N2 * 12 + kept * 12) / ms / 1e6
        T = perturb.UniformTransformSE3(20, 0.5, "uniform", True)
        res["generate_transforms_64_us"] = timeit(lambda: T.generate_transforms(64), reps=20) * 1e3
    print({k: round(v, 4) for k, v in res.items()})


if __name__ == "__main__" and "stamps" not in sys.argv:
    main()


def fps_stamps():
    """Per-phase cycle split of the FPS register kernel (diagnostic build)."""
    import ctypes
    L = _lib.load()
    fn = L.hreg_debug_fps_stamps
    fn.restype = ctypes.c_int
    vp, i = ctypes.c_void_p, ctypes.c_int
    fn.argtypes = [i, i, i, vp, vp, vp, vp, vp]
    rng = np.random.default_rng(0)
    for n, m, weighted in ((16384, 1024, False), (1024, 512, True)):
        x = torch.from_numpy(rng.uniform(-40, 40, (16, n, 3)).astype(np.float32)).cuda()
        w = torch.from_numpy(rng.uniform(0.5, 2, (16, n)).astype(np.float32)).cuda() if weighted else None
        idx = torch.empty((16, m), dtype=torch.int32, device="cuda")
        st = torch.zeros(8, dtype=torch.int64, device="cuda")
        for _ in range(2):
            rc = fn(16, n, m, x.data_ptr(), w.data_ptr() if w is not None else None, idx.data_ptr(),
                    st.data_ptr(), _lib.stream_handle())
            assert rc == 0
        torch.cuda.synchronize()
        s = st.cpu().numpy().astype(float)
        it = m - 1
        print(f"n={n} m={m}: cycles/iter scan={s[0]/it:.0f} wavered+pick={s[1]/it:.0f} "
              f"lds+barrier={s[2]/it:.0f} final={s[3]/it:.0f} total={s[4]/it:.0f}; "
              f"clock={s[4] / (s[5] / 100e6) / 1e9:.3f} GHz, {s[5] / 100e6 * 1e3:.3f} ms")


if __name__ == "__main__" and "stamps" in sys.argv:
    fps_stamps()
