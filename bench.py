"""Benchmark: point-cloud pairs/sec of the HRegNet forward (BASELINE.json metric).

Workload (BASELINE.json configs[1]): HRegNet forward, batch = 8 pairs per GPU,
2 x 16384-point KITTI-shape synthetic LiDAR pairs (pcd_reg_hregnet_amd.synthetic),
eval mode, fp32, weights = nusc_feats (pretrained feature extractor) + seeded
heads.  A step = one forward over one batch; inputs are resident in HBM before
the timed region.  Multi-GPU: one process per GPU, each rank runs its own 8
pairs (pairs are independent in eval mode: no collective on the data path),
weak scaling; value = all pairs / max-over-ranks time.

Extra fields: ``roofline`` for the dominant kernel family (the fp32 MFMA GEMM,
timed live with HIP events on the launch stream inside the timed region) and
``cpu_baseline`` (the CPU oracle restatement on the host cores, bounded sample,
rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: Peak FP32 (matrix)
PEAK_BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: Peak BF16 MFMA, dense
# fp32-accurate products on the bf16 matrix cores (bf16x6, mfma_chain.h): 6 bf16 MFMAs of
# the same shape per fp32 product, so the fp32-equivalent peak is the bf16 dense peak / 6
PEAK_B6_TFLOPS = PEAK_BF16_MFMA_TFLOPS / 6
PEAK_HBM_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E peak BW (spec)
# 20.51 GFLOP/pair of 1x1 convs (conv hooks on the reference) + 2 x 0.034
# GFLOP cosine-similarity contractions
ALG_GFLOP_PER_PAIR = 20.579
POINTS = 16384
PAIRS_PER_GPU = 8
LANES_MAX = 48         # graph executor: most batches in flight (memory: one forward's buffers each)
V2_POINTS = 65536      # config 5 (MANTruckScenes-shape): B=16 over 8 GPUs -> 2 pairs/GPU
V2_PAIRS_PER_GPU = 2
V2_LANES = 4           # Model_V2 graph executor: lanes (forwards in flight; 2 when --steps / merge is odd)
# Model_V2: reference batches merged per forward (--merge; the largest divisor of --steps up to
# this).  48 steps, paired lines (gpurun_out/r5p): merge 8 / 12 / 24 -> 2999 / 3164 / 3137 pairs/s
V2_MERGE = 12
# HRegNet line: reference batches of 8 pairs merged per executor forward (the largest divisor of
# --steps up to this).  Paired lines (one box, gpurun_out/r5m, r5p): --steps 20 on merge 1 / 2 /
# 4 / 5 / 10 / 20: 7391 / 7518 / 7797 / 7716 / 7768 / 6901 pairs/s; --steps 48 on 1 / 2 / 3 / 4 /
# 6 / 8: 7570 / 7969 / 7945 / 8029 / 7779 / 7672
HREGNET_MERGE = 4


class _Args:
    use_fps = True
    use_weights = True
    freeze_detector = False
    freeze_feats = False


def make_model(device, model="hregnet"):
    from pcd_reg_hregnet_amd import weights
    from pcd_reg_hregnet_amd.models import HRegNet, Model_V2
    net = (Model_V2 if model == "v2" else HRegNet)(_Args())
    net.load_state_dict(weights.make_state_dict(net.state_dict(), seed=0, pretrained_feats=True))
    return net.to(device).eval()


# Work per launch, as (algorithmic FLOPs, algorithmic bytes, executed FLOPs).  The
# algorithmic FLOPs are the reference's conv MACs x 2 (20.51 GFLOP/pair of
# 1x1 convs); executed FLOPs are what the MFMAs run: with the precomputed first-layer
# feature / descriptor blocks (engine.LEVEL_PRE, HEAD_PRE, COARSE_SPLIT) the products of
# a gathered or repeated block are made once per source row instead of once per grouped
# row, so fewer FLOPs execute than the reference's algorithm counts.
# level-1 fused kernel: per group 64 rows x (det 4*32+32*32+32*64, desc same,
# mlp1 192*32, mlp2 32*64) MACs = 64 * 14592 MAC (layers.py:115-121,183-198)
L1_FLOPS_PER_GROUP = 2.0 * 64 * (2 * (4 * 32 + 32 * 32 + 32 * 64) + 192 * 32 + 32 * 64)
# per group: geom 64 x float4 + knn_xyz 64 x 3 in, kp 3 + att_feat 64 + desc 64 out
L1_BYTES_PER_GROUP = 4.0 * (64 * 4 + 64 * 3 + 3 + 64 + 64)


def _level_flops(kn, cf, c1, c3, cm1, cm2, pre):
    """Fused level 2/3 kernel per group: kn rows x (det (4+cf)*c1 + c1*c1 + c1*c3, desc
    same, mlp1 3*c3*cm1, mlp2 cm1*cm2) MACs; pre: the cf-wide first-layer blocks precomputed."""
    cin = 4 if pre else 4 + cf
    return 2.0 * kn * (2 * (cin * c1 + c1 * c1 + c1 * c3) + 3 * c3 * cm1 + cm1 * cm2)


L2_FLOPS_PER_GROUP = _level_flops(32, 64, 64, 128, 64, 128, False)
L3_FLOPS_PER_GROUP = _level_flops(16, 128, 128, 256, 128, 256, False)
# bytes: geom kn x float4, knn_xyz kn x 3, gidx kn, gathered features kn x cf, out kp 3 +
# att_feat c3 + desc cm2
L2_BYTES_PER_GROUP = 4.0 * (32 * 4 + 32 * 3 + 32 + 32 * 64 + 3 + 128 + 128)
L3_BYTES_PER_GROUP = 4.0 * (16 * 4 + 16 * 3 + 16 + 16 * 128 + 3 + 256 + 256)


def _level_work(lvl):
    cfg = {2: (32, 64, 64, 128, 64, 128), 3: (16, 128, 128, 256, 128, 256)}[lvl]
    kn, cf, c1 = cfg[:3]
    nb = L2_BYTES_PER_GROUP if lvl == 2 else L3_BYTES_PER_GROUP

    def work(a):
        G, pre = a[5], a[9] is not None
        # pre: each row gathers its precomputed [det c1 | desc c1] row instead of the features
        b = nb + (4.0 * kn * (2 * c1 - cf) if pre else 0.0)
        return _level_flops(*cfg, False) * G, b * G, _level_flops(*cfg, pre) * G
    return work


def _fine_work(args):
    C, G = args[1], args[7]
    N1 = 2 * C  # conv MACs per row of 8 neighbours (unpadded); executed: with precomputed
    # descriptor products (engine.HEAD_PRE, args[10]) only the 12 small columns of convs_1[0]
    kx = 12 if args[10] is not None else 2 * C + 12
    return (2.0 * 8 * G * ((2 * C + 12) * N1 + 2 * N1 * N1),
            4.0 * G * (8 * (16 + C + 1 + 3) + C + 3 + N1),
            2.0 * 8 * G * (kx * N1 + 2 * N1 * N1))


def _fine6_work(args):
    """hreg_fine_head6 (table, C, small, gidx, knn_xyz, G, ...): precomputed blocks always"""
    C, G = args[1], args[5]
    N1 = 2 * C
    return (2.0 * 8 * G * ((2 * C + 12) * N1 + 2 * N1 * N1),
            4.0 * G * (8 * (16 + C + 1 + 3) + C + 3 + N1),
            2.0 * 8 * G * (12 * N1 + 2 * N1 * N1))


def _coarse6_work(args):
    """hreg_coarse_head6 (table, small, ud0, ud1, gidx, knn_xyz, G, ...): convs_1 over 8 G
    rows, 528 -> 512 -> 512 -> 512 (executed: the 16 small columns of the first layer)"""
    G = args[6]
    return (2.0 * 8 * G * (528 * 512 + 2 * 512 * 512), 4.0 * G * (8 * (16 + 512 + 3) + 512 + 512 + 3),
            2.0 * 8 * G * (16 * 512 + 2 * 512 * 512))


def _corr6_work(args):
    """hreg_corr_head6 (table, N1, small, ud0, ud1, gidx, knn_xyz, G, ...): FineReg convs_1
    over 8 G rows, (2C + 12) -> N1 -> N1 -> N1 with C = N1 / 2 (executed: the 12 small
    columns; N1 = 512 is CoarseReg's 528 -> 512 layers, 16 small columns)"""
    N1, G = args[1], args[7]
    kin = 528 if N1 == 512 else N1 + 12
    ks = 16 if N1 == 512 else 12
    return (2.0 * 8 * G * (kin * N1 + 2 * N1 * N1), 4.0 * G * (8 * (16 + N1 // 2 + 3) + N1 + 3 + N1),
            2.0 * 8 * G * (ks * N1 + 2 * N1 * N1))


def _nbr_work(args):
    G = args[4]
    kx = 4 if args[6] is not None else 260  # HEAD_PRE: geometry columns only
    return (2.0 * 8 * G * (260 * 256 + 2 * 256 * 256), 4.0 * G * (8 * (256 + 4 + 1) + 256),
            2.0 * 8 * G * (kx * 256 + 2 * 256 * 256))


def _mlp_work(args):
    C, G = args[1], args[4] * args[5]
    f = 2.0 * G * (2 * C * C + C)
    return f, 4.0 * G * (C + 1), f


def _l1_work(a):
    return L1_FLOPS_PER_GROUP * a[3], L1_BYTES_PER_GROUP * a[3], L1_FLOPS_PER_GROUP * a[3]


# C-ABI entry -> (timer kind, work of one launch from its arguments)
MFMA_ENTRIES = {
    "hreg_group_l1": ("level", _l1_work),
    "hreg_group_l1_6": ("level", _l1_work),
    "hreg_group_l1_6g": ("level", _l1_work),
    "hreg_group_l2": ("level", _level_work(2)),
    "hreg_group_l3": ("level", _level_work(3)),
    "hreg_group_split_l2": ("level", _level_work(2)),
    "hreg_group_split_l3": ("level", _level_work(3)),
    "hreg_group6_l2": ("level", _level_work(2)),
    "hreg_group_split6_l2": ("level", _level_work(2)),
    "hreg_group_split6_l3": ("level", _level_work(3)),
    "hreg_group_split6j_l3": ("level", _level_work(3)),
    "hreg_group6_l3": ("level", _level_work(3)),
    "hreg_fine_head": ("head", _fine_work),
    "hreg_nbr_head": ("head", _nbr_work),
    "hreg_fine_head6": ("head", _fine6_work),
    "hreg_nbr_head6": ("head", _nbr_work),
    "hreg_nbr_head6s": ("head", _nbr_work),
    "hreg_nbr_head6sx": ("head", _nbr_work),
    "hreg_coarse_head6": ("head", _coarse6_work),
    "hreg_corr_head6": ("head", _corr6_work),
    "hreg_corr_head6x": ("head", _corr6_work),
    "hreg_mlp_head": ("mlp", _mlp_work),
    "hreg_mlp_head6": ("mlp", _mlp_work),
    "hreg_mlp_head6x": ("mlp", _mlp_work),
}


class MfmaTimer:
    """Brackets every MFMA launch (gemm_nt_kernel, the fused level kernels, fine/nbr/mlp
    head kernels) with HIP events on the launch stream and counts its algorithmic FLOPs and
    bytes, per kernel kind and per C-ABI entry."""

    KINDS = ("gemm", "level", "head", "mlp")

    def __init__(self):
        self.events = {k: [] for k in self.KINDS}
        self.flops = dict.fromkeys(self.KINDS, 0.0)
        self.xflops = dict.fromkeys(self.KINDS, 0.0)
        self.bytes = dict.fromkeys(self.KINDS, 0.0)
        self.by_entry = {}  # C-ABI entry -> [(e0, e1)], algorithmic FLOPs
        self.enabled = False

    def _timed(self, kind, fn, flops, nbytes, xflops=None, entry=None):
        if not self.enabled:
            return fn()
        st = torch.cuda.current_stream()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st)
        r = fn()
        e1.record(st)
        self.events[kind].append((e0, e1))
        if entry is not None:
            ev, fl = self.by_entry.get(entry, ([], 0.0))
            ev.append((e0, e1))
            self.by_entry[entry] = (ev, fl + flops)
        self.flops[kind] += flops
        self.xflops[kind] += flops if xflops is None else xflops
        self.bytes[kind] += nbytes
        return r

    def install(self):
        from pcd_reg_hregnet_amd import _lib, engine
        orig_gemm, orig_gemm6 = _lib.gemm, _lib.gemm6
        orig_call = engine.call

        def gemm_of(fn, entry):
            def gemm(g):
                # algorithmic bytes: the A operand as presented (R x K, gathered rows
                # counted once per use), W and the output, fp32
                nbytes = 4.0 * g.batch * (g.R * g.K + g.N * g.K + g.R * g.N)
                return self._timed("gemm", lambda: fn(g), 2.0 * g.R * g.N * g.K * g.batch,
                                   nbytes, entry=entry)
            return gemm

        def call(name, *args):
            if name in MFMA_ENTRIES:
                kind, work = MFMA_ENTRIES[name]
                fl, nb, xf = work(args)
                return self._timed(kind, lambda: orig_call(name, *args), fl, nb, xf, entry=name)
            return orig_call(name, *args)
        orig_grouped = _lib.gemm_grouped

        def gemm_grouped(gs):
            fl = sum(2.0 * g.R * g.N * g.K * g.batch for g in gs)
            nb = sum(4.0 * g.batch * (g.R * g.K + g.N * g.K + g.R * g.N) for g in gs)
            return self._timed("gemm", lambda: orig_grouped(gs), fl, nb, entry="hreg_gemm_grouped")
        _lib.gemm = gemm_of(orig_gemm, "hreg_gemm")
        _lib.gemm6 = gemm_of(orig_gemm6, "hreg_gemm6")
        _lib.gemm_grouped = gemm_grouped
        engine.call = call

    def result(self, kind):
        torch.cuda.synchronize()
        ev = self.events[kind]
        ms = sum(a.elapsed_time(b) for a, b in ev)
        return ms, len(ev), self.flops[kind], self.bytes[kind], self.xflops[kind]

    def entries(self, steps):
        """per C-ABI entry: launches per step, mean launch duration, algorithmic TFLOP/s,
        the entry's MFMA peak (bf16x6 entries end in 6)"""
        torch.cuda.synchronize()
        out = {}
        for name, (ev, fl) in sorted(self.by_entry.items()):
            ms = sum(a.elapsed_time(b) for a, b in ev)
            out[name] = {"launches_per_step": round(len(ev) / max(steps, 1), 3),
                         "avg_launch_us": round(ms / max(len(ev), 1) * 1e3, 2),
                         "tflops": round(fl / max(ms, 1e-9) / 1e9, 2),
                         "peak": entry_peak(name), "_ms": ms, "_flops": fl}
        return out


def entry_peak(name: str) -> float:
    """MFMA peak (fp32-equivalent TFLOP/s) of a C-ABI entry's kernel: bf16x6 kernels
    (hreg_group_l1_6, hreg_group6_*, hreg_group_split6_*, hreg_*_head6) run on the bf16
    matrix cores, the others on v_mfma_f32_32x32x2_f32.  (r3: a suffix rule missed
    hreg_group_split6j_l3 / hreg_corr_head6x / hreg_nbr_head6sx and priced them at the fp32
    peak, inflating roofline.frac; tests/test_host_logic.py pins every entry's peak.)"""
    b6 = re.search(r"(l1_6|group6|split6|head6|gemm6)", name) is not None
    return PEAK_B6_TFLOPS if b6 else PEAK_FP32_MFMA_TFLOPS


def level_kernel(engine, lv: int) -> str:
    """rocprof name of the fused level kernel the engine's switches select."""
    if lv == 1:
        return "group_l1_6_kernel" if engine.B6_L1 else "group_l1_kernel"
    split = engine.SPLIT_L2 if lv == 2 else engine.SPLIT_L3
    b6 = engine.B6_L2 if lv == 2 else engine.B6_L3
    if split:
        if b6 and lv == 3 and engine.SPLIT_JT and engine.LEVEL_PRE:
            return "group_split6j_kernel"  # two row tiles per workgroup (csrc/group_split6.hip)
        return "group_split6_kernel" if b6 else "group_split_kernel"
    return "group_fused6_kernel" if b6 else "group_fused_kernel"


def pmc_traffic(kernel: str, workload: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes of THIS
    workload (the Model_V2 line had borrowed the 16384-point pass):
    profiles/r*_traffic.json keyed by workload ("hregnet:b8:n16384", "v2:b2:n65536:m8" -- m: reference
    batches merged per launch; made by
    tools/rocpd_summary.py traffic ... --key); the r1-r4 files hold the configs[1] pass alone.
    The latest round that measured every kernel of the family; (None, None) when no pass of
    this workload exists."""
    names = [n.split(" (")[0] for n in kernel.split(" + ")]
    for rnd in ("r6", "r5", "r4", "r3", "r2", "r1"):
        path = os.path.join(REPO, "profiles", f"{rnd}_traffic.json")
        try:
            d = json.load(open(path))
            if workload in d:
                d = d[workload]
            elif "bytes_per_launch" not in d or workload != "hregnet:b8:n16384":
                continue
            per = d["bytes_per_launch"]
            # one launch of each per step: mean over the family
            return sum(per[n] for n in names) / len(names), os.path.relpath(path, REPO)
        except (OSError, KeyError, ValueError):
            continue
    return None, None


def cpu_baseline(budget_s: float = 30.0, batches=(1, PAIRS_PER_GPU), reps: int = 3, v2: bool = False):
    """The oracle (numpy BLAS + the OpenMP C restatement of FPS / kNN, oracle/) on the host
    cores, timed as BASELINE.md section 4 asks: the same synthetic pairs as the GPU run at
    B=1 and B=8 (Model_V2: B=1 and 2 at 65536 points), 1 warm-up, median of `reps` runs each
    (time.perf_counter).  value = the largest batch's median (the GPU line's workload); a batch
    size whose runs would overrun the budget (estimated from the B=1 time) is skipped and named
    in `sample`."""
    from oracle import oracle
    from pcd_reg_hregnet_amd import synthetic, weights
    from pcd_reg_hregnet_amd.models import HRegNet, Model_V2
    points = V2_POINTS if v2 else POINTS
    sd = {k: v.numpy() for k, v in
          weights.make_state_dict((Model_V2 if v2 else HRegNet)(_Args()).state_dict(), seed=0).items()}
    s, d, _, _ = synthetic.lidar_batch(max(batches), points, seed0=0)

    def fwd(B):
        if v2:  # (the prime shuffles: fixed permutations; their draw is not the measured work)
            perm = np.roll(np.arange(B), 1)
            return oracle.model_v2_forward(sd, s[:B], d[:B], perm, perm)
        return oracle.hregnet_forward(sd, s[:B], d[:B])
    fwd(1)  # warm-up
    t_start = time.perf_counter()
    per_b, med = {}, {}
    for B in batches:
        if med and (time.perf_counter() - t_start) + reps * B * max(med.values()) > budget_s:
            continue
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fwd(B)
            ts.append(time.perf_counter() - t0)
        med[B] = float(np.median(ts)) / B  # s per pair
        per_b[f"B={B}"] = {"pairs_per_s": round(1.0 / med[B], 4),
                           "s_per_batch_median": round(float(np.median(ts)), 3),
                           "runs_s": [round(t, 3) for t in ts]}
    best_b = max(med)
    threads = int(oracle.lib().oracle_num_threads())
    # cores = the CPUs the oracle actually ran on: its OpenMP / BLAS threads, bounded by the
    # CPUs this process may be scheduled on (its affinity mask; os.cpu_count() is the whole
    # host's count, 256 on the GPU box)
    affinity = len(os.sched_getaffinity(0))
    return {"value": round(1.0 / med[best_b], 4), "unit": "pairs/s",
            "cores": min(threads, affinity), "omp_threads": threads, "affinity_cpus": affinity,
            "host_cpus": os.cpu_count(), "kind": "port", "batch": best_b, "per_batch": per_b,
            "sample": f"{'Model_V2' if v2 else 'HRegNet'} forward on 2x{points}-pt KITTI-shape "
                      f"synthetic LiDAR pairs (the GPU run's generator), B in {sorted(med)}, 1 "
                      f"warm-up + median of {reps} each; numpy BLAS + OpenMP C oracle (oracle/); value at B="
                      f"{best_b}; {threads} OpenMP/BLAS threads = OMP_NUM_THREADS as the GPU box "
                      "sets it: the box's CPU share per GPU (the host's other CPUs serve the "
                      "other GPUs' jobs; affinity_cpus is the whole mask); reference Python on 8 "
                      "vCPU (SURVEY container, BASELINE.md section 2): 0.55 pairs/s at B=1, "
                      "0.50 at B=8"}


def _fps_level(pts, m, weights, floor_call, floor_pts, floor_w, kernel):
    """one FPS level: the product kernel's launch time (HIP events) per dependent iteration,
    its s_memtime phase stamps (cloud 0's workgroup), and the floor geometry's stamps"""
    from pcd_reg_hregnet_amd import _lib
    nb, n, _ = pts.shape
    st_ = _lib.stream_handle()
    idx = torch.empty(nb, m, dtype=torch.int32, device=pts.device)
    temp = torch.full((nb, n), 1e10, device=pts.device)  # (the initial running minima, models/utils.py:25)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    name = "hreg_weighted_furthest_point_sampling" if weights is not None else "hreg_furthest_point_sampling"
    args = (nb, n, m, pts, weights, temp, idx, None, st_) if weights is not None else \
        (nb, n, m, pts, temp, idx, None, st_)
    if floor_call is None:  # the multi-workgroup kernel as the batched stage 1 launches it
        name, args = "hreg_fps_bounded", (nb, n, m, pts, temp, idx, None, 1, st_)
    _lib.call(name, *args)  # warm
    ev[0].record()
    _lib.call(name, *args)
    ev[1].record()
    if floor_call is None:  # (clouds above 16384 points: the multi-workgroup cluster kernel)
        torch.cuda.synchronize()
        launch_us = ev[0].elapsed_time(ev[1]) * 1e3
        return {"kernel": kernel, "clouds": nb, "points": n, "dependent_iterations": m - 1,
                "launch_us": round(launch_us, 1), "us_per_iteration": round(launch_us / (m - 1), 4)}
    stamps = torch.zeros(6, dtype=torch.int64, device=pts.device)
    _lib.call("hreg_debug_fps_stamps", nb, n, m, pts, weights, idx, stamps, st_)
    floor = torch.zeros(6, dtype=torch.int64, device=pts.device)
    fidx = torch.empty(nb, m, dtype=torch.int32, device=pts.device)
    floor_call(floor_pts, floor_w, fidx, floor, st_)
    torch.cuda.synchronize()
    scan, pick, barrier, final, total, ticks = [int(x) for x in stamps.cpu()]
    f_total, f_ticks = int(floor[4]), int(floor[5])
    ghz = total / (ticks * 10.0) if ticks else 0.0  # s_memrealtime: 100 MHz
    per_iter = lambda c, g=ghz: round(c / max(g, 1e-9) / 1e3 / (m - 1), 4)  # noqa: E731
    f_ghz = f_total / (f_ticks * 10.0) if f_ticks else 0.0
    launch_us = ev[0].elapsed_time(ev[1]) * 1e3
    return {"kernel": kernel, "clouds": nb, "points": n, "dependent_iterations": m - 1,
            "launch_us": round(launch_us, 1),
            "us_per_iteration": round(launch_us / (m - 1), 4),
            "stamped_us_per_iteration": per_iter(total),
            "stamped_scan_us_per_iteration": per_iter(scan),
            "stamped_exchange_us_per_iteration": per_iter(pick + barrier + final),
            "stamped_pick_us": per_iter(pick), "stamped_barrier_us": per_iter(barrier),
            "stamped_final_us": per_iter(final),
            "floor_us_per_iteration": per_iter(f_total, f_ghz),
            "frac_floor_over_kernel": round(per_iter(f_total, f_ghz) / max(per_iter(total), 1e-9), 3),
            "clock_ghz": round(ghz, 3)}


def _fps_sorted_level(pts, m, reg):
    """level 1 as the engine runs it with FPS_SORTED: the spatial index, then the FPS over its
    Morton-sorted copy with exact group pruning (hreg_fps_indexed), each timed with HIP events;
    the floor is the unstamped level-1 floor kernel (hreg_debug_fps_floor without stamps), timed
    the same way, so kernel and floor are compared unstamped.  reg: the register kernel's entry
    (its stamped phases), kept beside it."""
    from pcd_reg_hregnet_amd import _lib, engine
    nb, n, _ = pts.shape
    st_ = _lib.stream_handle()
    ws = torch.empty(engine.spatial_index_bytes(nb, n), dtype=torch.uint8, device=pts.device)
    idx = torch.empty(nb, m, dtype=torch.int32, device=pts.device)
    fp = pts[:, :1024].contiguous()
    fidx = torch.empty(nb, m, dtype=torch.int32, device=pts.device)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    for rep in range(2):  # (the first pass warms up)
        ev[0].record()
        _lib.call("hreg_spatial_index", pts, nb, n, ws, st_)
        ev[1].record()
        _lib.call("hreg_fps_indexed", nb, n, m, pts, ws, None, idx, None, st_)
        ev[2].record()
        _lib.call("hreg_debug_fps_floor", nb, m, fp, fidx, None, st_)
        ev[3].record()
    torch.cuda.synchronize()
    index_us = ev[0].elapsed_time(ev[1]) * 1e3
    launch_us = ev[1].elapsed_time(ev[2]) * 1e3
    floor_us = ev[2].elapsed_time(ev[3]) * 1e3
    per = lambda us: round(us / (m - 1), 4)  # noqa: E731
    if n > engine.FPS_SORTED_N:  # Model_V2's clouds: no floor kernel of this geometry
        return {"kernel": "fps_blocks_kernel (level 1: one 1024-thread workgroup per cloud, running "
                          "minima in registers, only the 64-point index blocks the new centre can change "
                          "read from the spatial index's sorted copy; hreg_fps_indexed)",
                "clouds": nb, "points": n, "dependent_iterations": m - 1,
                "index_us": round(index_us, 1), "launch_us": round(launch_us, 1),
                "us_per_iteration": per(launch_us),
                "basis": "HIP events around the index and the FPS launch", "cluster_kernel": reg}
    return {"kernel": "fps_sorted_kernel (level 1: 512 threads x 32 points of the spatial index's "
                      "Morton-sorted copy, 256-point groups skipped when their box cannot change them; "
                      "hreg_fps_indexed, engine.FPS_SORTED)",
            "clouds": nb, "points": n, "dependent_iterations": m - 1,
            "index_us": round(index_us, 1), "launch_us": round(launch_us, 1),
            "us_per_iteration": per(launch_us),
            "floor_us_per_iteration": per(floor_us),
            "frac_floor_over_kernel": round(floor_us / max(launch_us, 1e-9), 3),
            "basis": "unstamped kernel and unstamped floor kernel launch times (HIP events)",
            "reg_kernel": reg}


def fps_latency(src, dst):
    """The FPS chain of one forward (latency-bound, 1023 + 511 + 255 dependent
    iterations) against measured latency floors, on the batch's 2B
    clouds, per level:
    * the product kernel's launch time (HIP events) per dependent iteration;
    * the same kernel with s_memtime stamps around each phase of every iteration (cloud 0's
      workgroup): the distance scan vs the exchange (wave max + winner pick, LDS hand-off +
      barrier, block max);
    * the floor: the same workgroup and per-iteration exchange with (almost) no scan --
      level 1: 2 instead of 32 points per thread (hreg_debug_fps_floor); levels 2 / 3 (WFPS on
      1024 / 512 points): one weighted point per thread in the level's one-wave geometry
      (hreg_debug_wfps_floor), i.e. the dependent chain alone.
    Levels 2 / 3 run on the first 1024 / 512 points of each cloud with seeded weights in
    [0.5, 2] (the WFPS cost does not depend on the values)."""
    from pcd_reg_hregnet_amd import _lib
    pts = torch.cat([src, dst], 0).contiguous()
    nb = pts.shape[0]
    g = torch.Generator(device="cpu").manual_seed(5)
    out = {"basis": "floor = the same workgroup and per-iteration exchange with (almost) no "
                    "scan; stamped figures carry the s_memtime overhead on both sides"}
    if pts.shape[1] <= 16384:
        out["level1"] = _fps_level(
            pts, 1024, None,
            lambda fp, fw, i, s, st: _lib.call("hreg_debug_fps_floor", nb, 1024, fp, i, s, st),
            pts[:, :1024].contiguous(), None,
            "fps_reg_kernel<512, 2, 16> (level 1: 512 threads x 32 points per cloud)")
        from pcd_reg_hregnet_amd import engine
        if engine.FPS_SORTED and pts.shape[1] == engine.FPS_SORTED_N:
            out["level1"] = _fps_sorted_level(pts, 1024, out["level1"])
    else:  # Model_V2's 65536-point clouds
        out["level1"] = _fps_level(pts, 1024, None, None, None, None,
                                   "fps_cluster_kernel (level 1: one cloud over single-wave "
                                   "workgroups exchanging candidates through L2; hreg_fps_bounded, "
                                   "one launch at a time, as the r5 batched stage 1 ran it)")
        from pcd_reg_hregnet_amd import engine
        if engine.FPS_SORTED and engine.fps_indexed_ok(pts.shape[1]):
            out["level1"] = _fps_sorted_level(pts, 1024, out["level1"])
    for lvl, n, m, T, kern in ((2, 1024, 512, 64, "fps_reg_kernel<64, 16, 1, weighted> (level 2: 1 wave x 16 points, "
                                                  "fps.hip HREG_FPS_W1024_1W)"),
                               (3, 512, 256, 64, "fps_reg_kernel<64, 8, 1, weighted> (level 3: 1 wave x 8 points)")):
        p = pts[:, :n].contiguous()
        w = (0.5 + 1.5 * torch.rand(nb, n, generator=g)).to(pts.device)
        fp = pts[:, :T].contiguous()
        fw = w[:, :T].contiguous()
        out[f"level{lvl}"] = _fps_level(
            p, m, w,
            lambda fp_, fw_, i, s, st, T=T, m=m: _lib.call("hreg_debug_wfps_floor", nb, T, m, fp_, fw_, i, s, st),
            fp, fw, kern)
    out["chain_us"] = round(sum(out[f"level{k}"]["launch_us"] for k in (1, 2, 3))
                            + out["level1"].get("index_us", 0.0), 1)
    # (the r4 lines' flat fields: level 1)
    for k in ("us_per_iteration", "frac_floor_over_kernel", "floor_us_per_iteration",
              "stamped_us_per_iteration"):
        if k in out["level1"]:
            out[k] = out["level1"][k]
    return out


def forward_latency(P, src, dst, reps: int = 7, v2: bool = False):
    """Single-batch latency (the reference's callers run one batch at a
    time, test/test_v3.py:82,120): one batch-B forward alone on the device, median of `reps`
    after 2 warm-ups, (a) launched eagerly (engine.hregnet_forward, host launches) and (b) as
    the captured graph of a 1-lane GraphPipeline (stage 1 + the rest, two replays); both with
    engine.chain_fork's side-stream forks (the 1-lane GraphPipeline enables them itself)."""
    from pcd_reg_hregnet_amd import engine

    def med(fn):
        ts = []
        for i in range(reps + 2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            if i >= 2:
                ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e3
    def eager_forward():
        with engine.chain_fork():  # (the spatial index / level input projections beside the chain)
            out = engine.hregnet_forward(P, src, dst, v2=v2)
            if v2:
                engine.model_v2_finish(out)
    with torch.no_grad():
        eager = med(eager_forward)
        gp = engine.GraphPipeline(P, src, dst, lanes=1, v2=v2)
        graph = med(lambda: gp.run_forwards(1))
        del gp
    B = src.shape[0]
    return {"batch": B, "eager_ms": round(eager, 3), "graph_ms": round(graph, 3),
            "pairs_per_s_alone": round(B / graph * 1e3, 1),
            "basis": f"one batch of {B} pairs alone on the GPU, median of {reps} (synchronised); "
                     "graph = 1-lane GraphPipeline (stage-1 graph + rest-of-forward graph)"}


def unmerged_line(P, src, dst, steps: int, warmup: int):
    """the same timed steps with ONE reference batch of B pairs per executor forward
    (merge 1, steps lanes up to LANES_MAX: the r4 configuration), timed like the headline line
    (streamed rounds, primed, synchronised) -- reported beside the merged value, never as it."""
    from pcd_reg_hregnet_amd import engine
    B = src.shape[0]
    lanes = steps if steps <= LANES_MAX else max([d for d in range(16, LANES_MAX + 1) if steps % d == 0]
                                                   or [LANES_MAX])
    with torch.no_grad():
        gp = engine.GraphPipeline(P, src, dst, lanes=lanes)
        gp.prepare(warmup)
        gp.prepare(steps)
        gp.run_forwards(warmup, stream=True)
        gp.prime()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gp.run_forwards(steps, stream=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        del gp
    return {"value": round(B * steps / el, 3), "ms_per_step": round(el / steps * 1e3, 3), "lanes": lanes,
            "basis": f"the same {steps} timed batches of {B} pairs with one reference batch per executor "
                     f"forward ({lanes} forwards in flight), measured right after the headline line"}


def default_merge(steps: int, v2: bool, batch: int = PAIRS_PER_GPU) -> int:
    """Reference batches merged per executor forward when --merge is not given: the largest
    divisor of --steps up to the model's factor (HREGNET_MERGE / V2_MERGE), so any step count
    still times exactly --steps batches.  A batch of 32 pairs or more (configs[2]) already fills
    the chip: one batch per forward (r6, --steps 20, one box: merge 1 / 2 / 4 at B = 32 ran 8555 /
    8675 / 8502 pairs/s, gpurun_out/r6b32)."""
    cap = V2_MERGE if v2 else (HREGNET_MERGE if batch < 32 else 1)
    return max(m for m in range(1, cap + 1) if steps % m == 0) if steps > 0 else 1


def in_executor(steps: int, B: int, points: int, entries_flops: dict, merge: int = 1):
    """roofline of the level family inside the timed graph executor: the
    level kernels' mean durations over the timed region's dispatches, from the committed
    rocprofv3 kernel trace of `bench.py --steps S --warmup W --no-eager-roofline`
    (tools/in_executor.py -> profiles/r*_in_executor.json, keyed by workload), against the
    same algorithmic FLOPs per launch as the eager figure.  None when no trace of this
    workload is committed (key: batch, points, timed steps and merge factor; the timed region
    holds steps / merge launches of each level kernel)."""
    key = f"hregnet:b{B}:n{points}:s{steps}" + (f":m{merge}" if merge > 1 else "")
    for rnd in ("r6", "r5"):
        path = os.path.join(REPO, "profiles", f"{rnd}_in_executor.json")
        try:
            d = json.load(open(path))[key]
        except (OSError, KeyError, ValueError):
            continue
        if not isinstance(d, dict) or not isinstance(d.get("avg_us"), dict):
            continue    # malformed entry: no in-executor figure rather than no bench line
        t = 0.0
        fl = 0.0
        per = {}
        for kern, us in d["avg_us"].items():
            f = entries_flops.get(kern)
            if f is None:
                return None
            per[kern] = {"avg_us": us, "tflops": round(f / us / 1e6, 2)}
            t += us
            fl += f
        ach = fl / t / 1e6
        out = {"achieved": round(ach, 3), "frac": round(ach / PEAK_B6_TFLOPS, 4),
               "basis": "one launch of each level kernel: FLOPs over the sum of their mean "
                        "in-executor durations (each kernel shares the chip with the round's "
                        "other lanes, so this under-states the family's rate)",
               "per_kernel": per, "source": os.path.relpath(path, REPO),
               "dispatches": d.get("dispatches"), "tree": d.get("tree")}
        if d.get("union_us"):
            # every timed launch's FLOPs over the time any of them was running
            ach_u = fl * d["dispatches"] / d["union_us"] / 1e6
            out.update({"achieved_union": round(ach_u, 3), "frac_union": round(ach_u / PEAK_B6_TFLOPS, 4),
                        "union_us": d["union_us"]})
        return out
    return None


def provenance() -> dict:
    """HREG_SWITCHES / HREG_LIB of this run, and the timing probes among them (a line with
    probes is marked: it is not a measurement)"""
    from pcd_reg_hregnet_amd import switches
    out = switches.provenance()
    if switches.probes():
        out["PROBES_ACTIVE_NOT_A_MEASUREMENT"] = switches.probes()
    return out


def shard_batch(rank: int, pairs: int, points: int):
    """Rank r's own pairs (seeded by rank: shards are disjoint, no data exchange)."""
    from pcd_reg_hregnet_amd import synthetic
    return synthetic.lidar_batch(pairs, points, seed0=1000 * rank)


def max_over_ranks(elapsed: float, device) -> float:
    """The job's time = the slowest rank's (the only collective: one scalar, after timing)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return elapsed
    t = torch.tensor([elapsed], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def job_throughput(pairs_per_rank: int, steps: int, world: int, elapsed_max: float):
    """value = pairs processed by ALL ranks / max-over-ranks wall time (weak scaling)."""
    return pairs_per_rank * steps * world / elapsed_max


class TrainGemmTimer:
    """HIP events around every fp32-MFMA GEMM of the training step: the forward and
    input-gradient GEMMs (hreg_gemm -> gemm_nt_kernel) and the weight-gradient GEMMs
    (hreg_gemm_tn -> gemm_tn_kernel + split reduction), with their algorithmic FLOPs."""

    def __init__(self):
        self.ev = {"nt": [], "tn": []}
        self.flops = {"nt": 0.0, "tn": 0.0}
        self.enabled = False

    def _timed(self, kind, fn, flops):
        if not self.enabled:
            return fn()
        st = torch.cuda.current_stream()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st)
        r = fn()
        e1.record(st)
        self.ev[kind].append((e0, e1))
        self.flops[kind] += flops
        return r

    def install(self):
        from pcd_reg_hregnet_amd import _lib
        orig_gemm, orig_call = _lib.gemm, _lib.call

        def gemm(g):
            return self._timed("nt", lambda: orig_gemm(g), 2.0 * g.R * g.N * g.K * g.batch)

        def call(name, *a):
            if name == "hreg_gemm_tn":
                return self._timed("tn", lambda: orig_call(name, *a), 2.0 * a[4] * a[5] * a[6])
            if name in ("hreg_ts_gemm", "hreg_ts_gemm_bn"):  # (A, lda, R, K, W, w_trans, N, ...)
                return self._timed("nt", lambda: orig_call(name, *a), 2.0 * a[2] * a[3] * a[6])
            return orig_call(name, *a)
        _lib.gemm, _lib.call = gemm, call

    def result(self, kind):
        torch.cuda.synchronize()
        ms = sum(a.elapsed_time(b) for a, b in self.ev[kind])
        return ms, len(self.ev[kind]), self.flops[kind]


def bench_train(args, world, rank, device):
    """BASELINE configs[3]: train_reg_v0 step, 8 pairs of 2 x 16384 points per rank
    (batch 64 over 8 GPUs), DDP gradient averaging over RCCL (one bucket all-reduce)."""
    from pcd_reg_hregnet_amd import trainer, weights
    from pcd_reg_hregnet_amd.models import HRegNet
    net = HRegNet(_Args())
    net.load_state_dict(weights.make_state_dict(net.state_dict(), seed=0, pretrained_feats=True))
    net = net.to(device)
    tr = trainer.Trainer(net, lr=1e-3, alpha=1.0)
    B = args.batch
    s, d, Rg, tg = shard_batch(rank, B, args.points)
    src, dst = torch.from_numpy(s).to(device), torch.from_numpy(d).to(device)
    gR, gt = torch.from_numpy(Rg).to(device), torch.from_numpy(tg).to(device)
    # the step replayed from captured HIP graphs (trainer.GraphTrainer; bitwise the eager
    # step, tests/test_gpu_train_capture.py); with world > 1 the bucket all-reduce (RCCL) is
    # captured inside the graph
    # With world > 1 the captured RCCL all-reduce path runs only when asked for
    # (--train-graph-ddp): its one hardware execution so far is the 1-rank test
    # (tests/test_gpu_train_ddp.py::test_graph_trainer_rccl_world1), so the default multi-GPU
    # line keeps the eager DDP step the earlier rounds measured.  step_path records which ran.
    graphed = not args.train_eager and (world == 1 or (args.train_graph_ddp and
                                                       dist.get_backend() == "nccl"))
    eager_tr = tr
    if graphed:
        gtr = trainer.GraphTrainer(tr, B, args.points)
        gtr.capture(src, dst, gR, gt)
        tr = gtr
    timer = TrainGemmTimer()
    timer.install()
    nxt = (src, dst)  # the next step's batch: its level-1 grouping overlaps this step
    for _ in range(args.warmup):
        tr.step(src, dst, gR, gt, next_batch=nxt)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timer.enabled = not graphed  # (HIP events cannot sit inside a replayed graph)
    t0 = time.perf_counter()
    losses = [tr.step(src, dst, gR, gt, next_batch=nxt)[0].clone() for _ in range(args.steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if graphed:
        # the GEMM family's HIP events from an instrumented eager pass of the same steps right
        # after the timed region (the eager step launches the same kernels)
        timer.enabled = True
        for _ in range(args.steps):
            eager_tr.step(src, dst, gR, gt, next_batch=nxt)
        torch.cuda.synchronize()
    timer.enabled = False
    elapsed = max_over_ranks(elapsed, device)
    value = job_throughput(B, args.steps, world, elapsed)
    if rank == 0:
        line = train_line(args, B=B, world=world, value=value, elapsed=elapsed,
                          losses=[float(x) for x in (losses[0], losses[-1])], nt=timer.result("nt"),
                          tn=timer.result("tn"), graphed=graphed)
        print(json.dumps(line), flush=True)


def train_line(args, *, B, world, value, elapsed, losses, nt, tn, graphed):
    """The training bench's JSON line from its measurements (no GPU work: assembled on the CPU
    by tests/test_host_logic.py).  nt / tn: TrainGemmTimer.result of the two GEMM families;
    losses: the first and last timed step's loss."""
    nt_ms, nt_n, nt_fl = nt
    tn_ms, tn_n, tn_fl = tn
    ach = (nt_fl + tn_fl) / max(nt_ms + tn_ms, 1e-9) / 1e9
    fam = {"ts_gemm_kernel / gemm_nt_kernel (forward + input gradients)": {
               "launches_per_step": nt_n // args.steps,
               "ms_per_step": round(nt_ms / args.steps, 3),
               "tflops": round(nt_fl / max(nt_ms, 1e-9) / 1e9, 2)},
           "gemm_tn_kernel + tn_reduce (weight gradients)": {
               "launches_per_step": tn_n // args.steps,
               "ms_per_step": round(tn_ms / args.steps, 3),
               "tflops": round(tn_fl / max(tn_ms, 1e-9) / 1e9, 2)}}
    line = {
        "metric": "point-cloud pairs/sec, HRegNet training step (train_reg_v0), "
                  "16384-pt pairs",
        "value": round(value, 3), "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (seeded KITTI-shape LiDAR pairs with their ground-truth SE(3); "
                "nusc_feats + seeded heads)",
        "config": {"workload": f"HRegNet train step (train-mode BN, 3-level "
                               f"transformation_loss, backward, Adam), batch={B} pairs/GPU, "
                               f"2x{args.points}-pt pairs (BASELINE configs[3])",
                   "global_batch": B * world, "points": args.points,
                   "parallelism": f"dp{world} (one 9.87 MB gradient all-reduce per step)"},
        "loss_first_last": [round(losses[0], 5), round(losses[-1], 5)],
        "executor": "HIP graphs (two captured steps, ping-pong inputs)" if graphed else "eager",
        "step_path": ("GraphTrainer (captured step" + (", RCCL all-reduce captured in the graph)"
                                                      if world > 1 else ", no collective at world 1)")
                      if graphed else "Trainer (eager step" + (
                          ", RCCL all-reduce launched eagerly)" if world > 1 else ")")),
        "provenance": provenance(),
        "roofline": {"kernel": "fp32 MFMA GEMM family of the step (forward, input- and "
                               "weight-gradient GEMMs)",
                     "timing": ("HIP events on the launch stream, instrumented eager pass of the "
                                "same steps after the timed region" if graphed else
                                "HIP events on the launch stream inside the timed region"),
                     "bound": "mfma", "achieved": round(ach, 3),
                     "peak": PEAK_FP32_MFMA_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(ach / PEAK_FP32_MFMA_TFLOPS, 4), "traffic": None,
                     "gemm_ms_per_step": round((nt_ms + tn_ms) / args.steps, 3),
                     "gflop_per_pair": round((nt_fl + tn_fl) / args.steps / B / 1e9, 3),
                     "families": fam},
        "cpu_baseline": None,
    }
    return line


def forward_line(args, *, v2, B, merge, world, value, ms_per_step, host_submit_s, res, ent, level_names,
                 traffic, inexec, fps, lat, cpu, bs1, fs, merge1=None):
    """The forward bench's JSON line from its measurements (no GPU work here: tests assemble it
    on the CPU from synthetic measurements, tests/test_host_logic.py).  res: MfmaTimer.result per
    kind; ent: MfmaTimer.entries; traffic: pmc_traffic's (bytes, source)."""
    def kind_summary(k):
        ms, n, fl, nb, xf = res[k]
        return {"launches_per_step": round(n / args.steps, 3),
                "avg_launch_us": round(ms / max(n, 1) * 1e3, 2),
                "ms_per_step": round(ms / args.steps, 3),
                "tflops": round(fl / max(ms, 1e-9) / 1e9, 2),
                "gflop_per_pair": round(fl / args.steps / B / 1e9, 3),
                "executed_tflops": round(xf / max(ms, 1e-9) / 1e9, 2),
                "executed_gflop_per_pair": round(xf / args.steps / B / 1e9, 3)}
    # roofline kernel family: the three fused level kernels (keypoint detector +
    # descriptor, levels 1-3), the largest MFMA family of the step
    f_ms, f_n, f_fl, f_nb, f_xf = res["level"]
    per_launch_s = f_ms / max(f_n, 1) / 1e3
    per_launch_flops = f_fl / max(f_n, 1)
    achieved = per_launch_flops / per_launch_s / 1e12 if per_launch_s > 0 else 0.0
    lev = {n: e for n, e in ent.items() if n in MFMA_ENTRIES and MFMA_ENTRIES[n][0] == "level"}
    # the family's peak: its FLOPs over the time they need at each kernel's own peak
    t_peak = sum(e["_flops"] / (e["peak"] * 1e12) for e in lev.values())
    peak = sum(e["_flops"] for e in lev.values()) / t_peak / 1e12 if t_peak else PEAK_B6_TFLOPS
    traffic, traffic_src = traffic
    tot_ms = sum(r[0] for r in res.values())
    tot_xf = sum(r[4] for r in res.values())
    alg_fl = ALG_GFLOP_PER_PAIR * 1e9 * B * args.steps
    per_entry = {n: {k: v for k, v in e.items() if not k.startswith("_")} for n, e in ent.items()}
    roof = {"kernel": " + ".join(level_names) + " (keypoint detector + descriptor of "
                      "levels 1-3: every conv/BN/ReLU layer, attention and k-max of a "
                      "level in one launch)",
            "timing": "HIP events on the launch stream, " + (
                "instrumented eager pipelined pass of the same steps after the timed "
                "graph region" if args.executor == "graph" else "inside the timed region"),
            "bound": "mfma", "achieved": round(achieved, 3), "peak": round(peak, 1),
            "unit": "TFLOP/s",
            "peak_basis": "fp32-accurate products: bf16x6 kernels at the bf16 dense MFMA "
                          f"peak / 6 = {PEAK_B6_TFLOPS:.1f}, fp32-MFMA kernels at "
                          f"{PEAK_FP32_MFMA_TFLOPS} (MI355X_MICROARCH.md); FLOP-weighted "
                          "over the family",
            "frac": round(achieved / peak, 4),
            "traffic": None if traffic is None else round(traffic),
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": round(f_nb / max(f_n, 1)),
            "flop_per_launch": round(per_launch_flops),
            "executed_flop_per_launch": round(f_xf / max(f_n, 1)),
            "executed_tflops": round(f_xf / max(f_ms, 1e-9) / 1e9, 3),
            "launches_per_step": round(f_n / args.steps, 3),
            "avg_launch_us": round(per_launch_s * 1e6, 2),
            "other_mfma_kernels": {"gemm_nt_kernel": kind_summary("gemm"),
                                   "fine/nbr head kernels": kind_summary("head"),
                                   "mlp_head_kernel": kind_summary("mlp")},
            "per_entry": per_entry,
            "all_mfma": {"ms_per_step": round(tot_ms / args.steps, 3),
                         "gflop_per_pair": ALG_GFLOP_PER_PAIR,
                         "tflops": round(alg_fl / max(tot_ms, 1e-9) / 1e9, 2),
                         "executed_gflop_per_pair": round(tot_xf / args.steps / B / 1e9, 3),
                         "executed_tflops": round(tot_xf / max(tot_ms, 1e-9) / 1e9, 2)}}
    if not v2 and args.executor == "graph":
        roof["in_executor"] = inexec
    # the whole timed step: every MFMA family's algorithmic FLOPs per pair x pairs/s
    roof["step_tflops"] = round(ALG_GFLOP_PER_PAIR * value / 1e3, 2)
    roof["step_frac"] = round(ALG_GFLOP_PER_PAIR * value / 1e3 / PEAK_B6_TFLOPS, 4)
    line = {
        "metric": ("point-cloud pairs/sec, Model_V2 forward, 65536-pt pairs (config 5)" if v2
                   else "point-cloud pairs/sec, HRegNet forward, 16384-pt pairs"),
        "value": round(value, 3), "unit": "pairs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
        "host_submit_ms": round(host_submit_s * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "precision": "fp32 throughout; the fused level and head kernels take their fp32 "
                     "products on the bf16 matrix cores as 3-piece exact splits (bf16x6, "
                     "6 MFMAs per product, fp32 accumulate: error vs fp64 equal to the "
                     "fp32 MFMA's, profiles/r2_split_mfma_micro.txt); parity tests at the "
                     "fp32 bars",
        "data": "synthetic (seeded KITTI-shape LiDAR pairs; nusc_feats + seeded heads)",
        "config": {"workload": (f"Model_V2 forward (eval), batch={B} pairs/GPU, 2x{args.points}"
                                "-pt LiDAR pairs (BASELINE configs[4])") if v2 else (
                               f"HRegNet forward (eval), batch={B} pairs/GPU, "
                               f"2x{args.points}-pt KITTI-shape pairs (BASELINE "
                               + ("configs[2]: 3-level coarse-to-fine + weighted SVD, MFMA similarity"
                                  if B == 32 else "configs[1]") + ")"),
                   "executor": args.executor + ("" if args.executor == "serial" else
                               " (level-1 FPS of step i+1 overlaps step i)") + (
                               f", {args.lanes} forwards in flight" if args.lanes > 1 and
                               args.executor == "graph" else "") + (
                               f"; {merge} batches of {B} pairs merged per forward (one launch "
                               "set, every batch's outputs bitwise its own forward's; per-batch "
                               "SVD fallback" + (" and prime shuffles" if v2 else "") + ")"
                               if merge > 1 else "") + (
                               "; batched stage 1 (the level-1 FPS -- fps_blocks_kernel, one workgroup per cloud -- "
                               "spatial index and kNN as one launch each over every lane's clouds)"
                               if bs1 and args.points > 16384 else "") + (
                               "; front streaming: each timed round runs the registration "
                               "half of its batches and the feature extraction of the next "
                               "round's (pipeline primed after the warm-up)"
                               if fs else ""),
                   "global_batch": B * world, "points": args.points, "merge": merge,
                   "parallelism": f"dp{world} (pairs sharded, no collective)"},
        "roofline": roof,
        "merge1": merge1,
        "fps": fps,
        "latency": lat,
        "cpu_baseline": cpu,
        "provenance": provenance(),
    }
    return line


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list[str]) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes of this script (one
    per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment) and wait for
    them.  Runs before anything touches the GPU in this process; exit code = the worst
    rank's.  (Under torchrun WORLD_SIZE is already set and no process is spawned.)"""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc]
    return bad[0] if bad else 0


def init_world(args):
    """-> (world, rank, local rank) of this process; initialises the process group for
    N > 1 and checks it holds exactly --gpus ranks."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        if args.backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.backend)
        live = dist.get_world_size()
        if live != args.gpus:
            raise SystemExit(f"bench: initialised world size {live} != --gpus {args.gpus}")
        world, rank = live, dist.get_rank()
    return world, rank, local


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")),
                    help="GPUs of this node, one rank each; without torchrun (WORLD_SIZE "
                         "unset) bench.py starts the N rank processes itself")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="process-group backend (nccl = RCCL; gloo only for --launch-check)")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks, initialise the process group, print each rank's "
                         "{rank, world} and exit (no GPU work; the CPU launcher test)")
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", choices=("hregnet", "v2", "train"), default="hregnet",
                    help="v2: Model_V2 at config 5 (2 x 65536-pt pairs per GPU); train: the "
                         "train_reg_v0 step at config 4 (8 pairs per GPU, DDP)")
    ap.add_argument("--batch", type=int, default=None,
                    help=f"pairs per GPU (default {PAIRS_PER_GPU}; {V2_PAIRS_PER_GPU} for v2)")
    ap.add_argument("--points", type=int, default=None,
                    help=f"points per cloud (default {POINTS}; {V2_POINTS} for v2)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--merge", type=int, default=None,
                    help="reference batches (of --batch pairs) per executor forward, one launch set "
                         f"(default: the largest divisor of --steps up to {HREGNET_MERGE}, {V2_MERGE} "
                         "for v2); a step is still one batch")
    ap.add_argument("--train-eager", action="store_true",
                    help="--model train: launch the step eagerly instead of replaying captured graphs")
    ap.add_argument("--train-graph-ddp", action="store_true",
                    help="--model train with --gpus > 1: replay the captured step with the RCCL "
                         "all-reduce inside the graph (default: the eager DDP step)")
    ap.add_argument("--no-eager-roofline", action="store_true",
                    help="skip the instrumented eager pass after the timed graph region (the "
                         "rocprofv3 trace run behind roofline.in_executor: the timed replays are "
                         "then the last level-kernel dispatches of the run)")
    ap.add_argument("--no-merge1", action="store_true",
                    help="skip the unmerged (one reference batch per forward) figure beside a merged line")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the single-batch latency entry")
    ap.add_argument("--allow-probes", action="store_true",
                    help="run with PROBE_* timing switches set (results change: the line is "
                         "marked as a probe, never a measurement)")
    ap.add_argument("--executor", choices=("graph", "pipeline", "serial"), default="graph",
                    help="graph: pipelined forward replayed as HIP graphs; pipeline: same "
                         "eagerly; serial: no cross-batch overlap")
    ap.add_argument("--lanes", type=int, default=None,
                    help="graph executor: batches in flight at once, one stream each "
                         "(a step is still one forward over one batch); default: --steps "
                         "up to 48 (one round), else its largest divisor in [16, 48]; 4 "
                         "for v2 (its cluster FPS spins up to 256 waves per launch and "
                         "needs every launch's participants co-resident).  An explicit "
                         "value that --steps does not divide: the most lanes that do")
    ap.add_argument("--cpu-budget", type=float, default=30.0)
    ap.add_argument("--split", default=None,
                    help="comma list of levels (2,3) on the channel-split group kernel "
                         "(default: the engine's SPLIT_L2/SPLIT_L3)")
    ap.add_argument("--layerwise", default="",
                    help="comma list of levels (1,2,3) to run layer by layer instead of fused")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.launch_check:
        # the bench's rank plumbing without GPU work: shard, max-over-ranks, throughput
        world, rank, _ = init_world(args)
        s, d, _, _ = shard_batch(rank, 1, 1024)
        el = max_over_ranks(0.5 + rank, torch.device("cpu"))
        print(json.dumps({"rank": rank, "world": world, "shard_sum": float(s.sum() + d.sum()),
                          "elapsed_max": el, "value": job_throughput(1, 10, world, el)}),
              flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    v2 = args.model == "v2"
    if args.batch is None:
        args.batch = V2_PAIRS_PER_GPU if v2 else PAIRS_PER_GPU
    if args.points is None:
        args.points = V2_POINTS if v2 else POINTS
    # --merge M: each forward of the executor runs M reference batches of
    # --batch pairs merged into one launch set (engine.hregnet_forward sub_batch: every pair's
    # result bitwise that of its own batch's forward, the weighted SVD's identity fallback and
    # the prime shuffles per batch); a step is still one batch of --batch pairs
    merge = default_merge(args.steps, v2, args.batch) if args.merge is None else args.merge
    if merge < 1 or args.steps % merge:
        raise SystemExit(f"bench: --steps {args.steps} is not a multiple of --merge {merge}")
    args.warmup = -(-args.warmup // merge) * merge  # (untimed: rounded up to whole forwards)
    steps_arg = args.steps
    args.steps //= merge  # forwards (of merged batches) from here on; restored for the line
    args.warmup //= merge
    lanes_auto = args.lanes is None
    if lanes_auto:
        # one round when it fits: a replay boundary drains the pipeline and the round's
        # level-1 stage runs once per round (batched over its lanes, GraphPipeline
        # BATCH_STAGE1): lanes = --steps up to LANES_MAX, else the largest divisor of --steps
        # in [16, LANES_MAX] (measured on one box: --steps 24 on 8 / 12 / 24 lanes 6122 /
        # 6295 / 6432 pairs/s; --steps 48 on 16 / 24 / 48 lanes 6802 / 6697 / 6891), else
        # LANES_MAX with a final partial round (GraphPipeline.run_forwards); v2: 4
        if v2:
            # (r6, --steps 48, gpurun_out/r6v2: 4 lanes x 12 merged 6646 pairs/s, 2 x 12 6329,
            # 2 x 24 6574, 8 x 6 6278, 4 x 6 5947)
            args.lanes = max(ln for ln in (V2_LANES, 2, 1) if args.steps % ln == 0)
        elif args.steps <= LANES_MAX:
            args.lanes = max(args.steps, 1)
        else:
            divs = [d for d in range(16, LANES_MAX + 1) if args.steps % d == 0]
            args.lanes = max(divs) if divs else LANES_MAX
    if (args.model != "train" and args.executor == "graph" and args.steps % args.lanes
            and not lanes_auto):
        # a replay runs one batch per lane: time exactly --steps forwards with the most
        # lanes <= --lanes that divide it, powers of two first (the streams share
        # GPU_MAX_HW_QUEUES = 4 hardware queues: 5 or 6 lanes measured slower than 4; a
        # final partial round on some lanes, GraphPipeline.run_forwards, measured slower
        # too: --steps 20 on 8 lanes 5179 vs 4 lanes 5293 pairs/s)
        cand = [d for d in range(1, args.lanes + 1) if args.steps % d == 0]
        pow2 = [d for d in cand if d & (d - 1) == 0]
        lanes = max(pow2) if max(pow2) >= 4 or max(pow2) == max(cand) else max(cand)
        print(f"bench: --steps {args.steps} is not a multiple of --lanes {args.lanes}; "
              f"using {lanes} lanes", file=sys.stderr)
        args.lanes = lanes
    from pcd_reg_hregnet_amd import switches
    if switches.probes() and not args.allow_probes:
        raise SystemExit(f"bench: timing probes {switches.probes()} are set in HREG_SWITCHES "
                         "(they skip or repeat work: no measurement); --allow-probes to run them")
    world, rank, local = init_world(args)
    device = torch.device("cuda", local)

    from pcd_reg_hregnet_amd import _lib, engine
    _lib.load()
    if args.model == "train":
        bench_train(args, world, rank, device)
        if world > 1:
            dist.destroy_process_group()
        return
    for lv in filter(None, args.layerwise.split(",")):
        setattr(engine, f"FUSED_L{int(lv)}", False)
    if args.split is not None:
        on = {int(x) for x in filter(None, args.split.split(","))}
        engine.SPLIT_L2, engine.SPLIT_L3 = 2 in on, 3 in on
    level_names = [level_kernel(engine, lv) + f" (level {lv})" for lv in (1, 2, 3)]
    net = make_model(device, args.model)
    P = net.prepared(device)
    B = args.batch
    s, d, _, _ = shard_batch(rank, B * merge, args.points)
    src = torch.from_numpy(s).to(device)
    dst = torch.from_numpy(d).to(device)
    sb = B if merge > 1 else None

    timer = MfmaTimer()
    timer.install()

    pipe = engine.Pipeline(P, device, v2=v2, sub_batch=sb)
    gpipe = None
    if args.executor == "graph":
        with torch.no_grad():
            gpipe = engine.GraphPipeline(P, src, dst, lanes=args.lanes, v2=v2, sub_batch=sb)
            gpipe.prepare(args.warmup)
            gpipe.prepare(args.steps)  # captured before the timed region

    def run(n):
        with torch.no_grad():
            if args.executor == "serial":
                if v2:
                    return [engine.model_v2_finish(engine.hregnet_forward(P, src, dst, v2=True, sub_batch=sb), sb)
                            for _ in range(n)]
                return [engine.hregnet_forward(P, src, dst, sub_batch=sb) for _ in range(n)]
            if args.executor == "graph":
                # a continuous stream of batches: each call's last replay also runs the next
                # round's batched stage 1, so the warm-up leaves the first timed round's
                # stage 1 done and the timed region runs exactly one stage 1 per round
                # (the next round's) beside its forwards, as in the steady state
                return gpipe.run_forwards(n, stream=True)
            return pipe.run([(src, dst)] * n)

    run(args.warmup)
    if gpipe is not None:
        # (front streaming, engine.GraphPipeline: fill the pipeline so that every timed round
        # runs the registration half of its batches and the feature extraction of the next
        # round's -- whole forwards per round, as the streamed stage 1 already is)
        with torch.no_grad():
            gpipe.prime()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # HIP events cannot be recorded inside a captured graph (hipErrorInvalidHandle),
    # so with the graph executor the MFMA kernels are timed in an instrumented eager
    # pipelined pass of the same K steps right after the timed region; rocprofv3 on
    # this script reports the graph-replayed kernels' durations for comparison.
    timer.enabled = args.executor != "graph"
    t0 = time.perf_counter()
    out = run(args.steps)
    host_submit_s = time.perf_counter() - t0  # the host's share: launches / replays submitted
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    merge1 = None
    if (merge > 1 and not v2 and world == 1 and args.executor == "graph" and not args.no_merge1):
        try:
            merge1 = unmerged_line(P, src[:B], dst[:B], args.steps * merge, args.warmup * merge)
        except Exception as e:  # a side figure must never sink the GPU number
            merge1 = {"error": repr(e)}
    if args.executor == "graph" and not args.no_eager_roofline:
        timer.enabled = True
        with torch.no_grad():
            pipe.run([(src, dst)] * args.steps)
        torch.cuda.synchronize()
    timer.enabled = False
    res = {k: timer.result(k) for k in MfmaTimer.KINDS}
    # per reference batch of B pairs from here on (a forward ran `merge` of them)
    args.steps, args.warmup = steps_arg, args.warmup * merge

    elapsed = max_over_ranks(elapsed, device)
    value = job_throughput(B, args.steps, world, elapsed)
    ms_per_step = elapsed / args.steps * 1e3

    if rank == 0:
        ent = timer.entries(args.steps)
        traffic = pmc_traffic(" + ".join(level_names), f"{args.model}:b{B}:n{args.points}"
                              + (f":m{merge}" if merge > 1 else ""))
        # level-kernel FLOPs per launch at this batch (groups = 2B clouds x the level's
        # keypoints), by rocprof kernel name: the in-executor figure's numerators
        # (a launch covers the `merge` batches of one executor forward)
        lv_fl = {level_kernel(engine, 1): L1_FLOPS_PER_GROUP * 2 * B * merge * engine.LEVELS[0][0],
                 level_kernel(engine, 2): L2_FLOPS_PER_GROUP * 2 * B * merge * engine.LEVELS[1][0],
                 level_kernel(engine, 3): L3_FLOPS_PER_GROUP * 2 * B * merge * engine.LEVELS[2][0]}
        inexec = None
        if not v2 and args.executor == "graph":
            try:
                inexec = in_executor(args.steps, B, args.points, lv_fl, merge)
            except Exception as e:  # a committed-trace figure must never sink the GPU number
                inexec = {"error": repr(e)}
        fps = None
        try:
            fps = fps_latency(src[:B], dst[:B])
        except Exception as e:  # a diagnostic must never sink the GPU number
            fps = {"error": repr(e)}
        lat = None
        if not args.no_latency:
            try:
                lat = forward_latency(P, src[:B], dst[:B], v2=v2)
            except Exception as e:  # a diagnostic must never sink the GPU number
                lat = {"error": repr(e)}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            try:
                cpu = (cpu_baseline(args.cpu_budget, batches=(1, V2_PAIRS_PER_GPU), v2=True) if v2
                       else cpu_baseline(args.cpu_budget))
            except Exception as e:  # the baseline must never sink the GPU number
                cpu = {"error": repr(e)}
        line = forward_line(args, v2=v2, B=B, merge=merge, world=world, value=value,
                            ms_per_step=ms_per_step, host_submit_s=host_submit_s, res=res, ent=ent,
                            level_names=level_names, traffic=traffic, inexec=inexec, fps=fps, lat=lat,
                            cpu=cpu, bs1=gpipe is not None and gpipe.bs1, fs=gpipe is not None and gpipe.fs,
                            merge1=merge1)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    del out


if __name__ == "__main__":
    main()
