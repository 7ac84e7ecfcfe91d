"""HRegNet forward on the HIP library: weight preparation + launch sequence.

This is the host side of the hot path (models/HRegNet/models.py:77-148).  It
holds no math of its own: every stage is one or more C-ABI launches
(include/hregnet_amd.h) on PyTorch's current stream; torch only provides
device memory.  Activations are point-major ([rows][channels]) in HBM, rows
ordered (cloud, keypoint, neighbour).  src and dst clouds run through the
feature extractor together (2B clouds per launch; the reference makes two
passes, models.py:79-80).

Weight preparation folds eval-mode BatchNorm into a per-channel affine epilogue
(y = acc * alpha + beta, alpha = gamma / sqrt(var + eps), beta = b - mean * alpha,
the same fold torch's CPU batch_norm uses), and permutes the input columns of
the correspondence heads so the GEMM reads one packed 16/12-float small-feature
segment followed by the two descriptor segments (the sum over channels is
order-independent up to fp32 rounding).
"""
from __future__ import annotations

import contextlib
from dataclasses import dataclass

import torch

from . import _lib, capture, switches
from ._lib import Gemm, Seg, call

BN_EPS = 1e-5

# (nsample, k, in_feat, det_channels, desc_channels, desc_dim) per level:
# models/HRegNet/models.py:14-24
LEVELS = (
    (1024, 64, 0, (32, 32, 64), (32, 32, 64), 64),
    (512, 32, 64, (64, 64, 128), (64, 64, 128), 128),
    (256, 16, 128, (128, 128, 256), (128, 128, 256), 256),
)
K_HEAD = 8  # CoarseReg/FineReg k (models.py:71-73)
# ---- the product path's kernel forms.  Plain attributes: the defaults ARE the product path; the
# alternatives are test checkers (the layer-by-layer GEMM paths, the fp32-MFMA twins in
# libhregnet_checkers.so, the unsplit / unfused forms), set by tests with monkeypatch.
FUSED_L1 = True  # level 1 through the fused group_l1 kernel (False: layer-by-layer GEMMs)
FUSED_L2 = True  # level 2 through the fused group_fused kernel (k = 32)
FUSED_L3 = True  # level 3 through the fused group_fused kernel (k = 16)
# levels 2 / 3 on the channel-split kernel (group_split6.hip) instead of the accumulator-chained
# one (group_fused6.hip); measured per level (r2-r3: level 3 split, level 2 chained + LDS ring)
SPLIT_L2 = False
SPLIT_L3 = True
SPLIT_JT = True  # level 3 on the two-row-tile form of the channel-split kernel (hreg_group_split6j_l3)
# 32-row tiles per workgroup of the channel-split FineReg / neighbour heads (0: the library's
# default, two at N1 <= 256; hreg_corr_head6x / hreg_nbr_head6sx)
HEAD_ROW_TILES = 0
# the fused kernels on the bf16 matrix cores at fp32 accuracy (bf16x6 split products) instead of
# their v_mfma_f32_32x32x2_f32 twins (checkers)
B6_L1 = B6_L2 = B6_L3 = True
B6_GEMM = True  # the big plain GEMMs (CoarseReg convs_1 layers 2-3) on hreg_gemm6
B6_MLP = True  # mlp heads on hreg_mlp_head6
B6_HEADS = True  # FineReg / CoarseReg-neighbour heads (group_head.hip *_head6_kernel)
FUSED_COARSE = True  # CoarseReg convs_1 (split first layer) + attention in one launch (coarse6.hip)
SPLIT_FINE = True  # FineReg heads on coarse6.hip's channel-split correspondence kernel
SPLIT_NBR = True  # the neighbour branch likewise
FUSED_FINE = True  # FineReg convs_1 + attention through group_head.hip
FUSED_NBR = True  # CoarseReg neighbour branch (convs_2 + attention) through group_head.hip
FUSED_HEAD = True  # mlp1 -> mlp2 -> mlp3 heads in one launch each (mlp_head.hip)
# CoarseReg convs_1[0] as [small] GEMM + per-keypoint desc / knn_desc products added in the
# epilogue (distributivity over the concatenation, layers.py:364-384; False: one 528-deep GEMM)
COARSE_SPLIT = True
# the same for the fused FineReg heads (descriptor blocks of convs_1[0]) and the CoarseReg
# neighbour branch (descriptor block of convs_2[0]): per-point products precomputed, the
# fused kernels multiply only the small / geometry columns per row
HEAD_PRE = True
# levels 2 / 3: the feature blocks of the detector's and the descriptor's first conv,
# W_f f per level-(l-1) feature row, precomputed once (one GEMM) instead of once per
# grouped row (k = 32 / 16 rows gather each feature row)
LEVEL_PRE = True
# level 1 with its weight table resident in LDS (hreg_group_l1_6) for clouds up to this many
# points; above, the global-table form (hreg_group_l1_6g): r2, beside Model_V2's cluster FPS on
# every CU the 92 KB LDS claim waited for it (942 vs 856 pairs/s)
L1_LDS_MAX_N = 16384  # (r6, beside the one-workgroup V2 FPS: 65536 measured within noise, 6407 / 6749 / 6517 vs 6329 / 6574 / 6646)

# ---- executor switches (HREG_SWITCHES, whole-process A/B of the measured choices)
# GraphPipeline: level-1 stage of all lanes as one batched launch per kernel (one side stream)
# instead of one per lane (r2: 5424 -> 6213 pairs/s)
BATCH_STAGE1 = switches.flag("BATCH_STAGE1", True)
V2_BATCH_STAGE1 = switches.flag("V2_BATCH_STAGE1", True)  # GraphPipeline(v2=True): see bs1
# GraphPipeline: halves of a forward in consecutive rounds, the two halves of a lane on two
# streams (r4: 20 lanes 7084 -> 7311 pairs/s; off above FRONT_STREAM_MAX_LANES: 48 lanes 7456 ->
# 7388; off for Model_V2: r6, 6142 / 6966 / 6423 vs 6329 / 6574 / 6646 pairs/s at 2 x 12, 2 x 24,
# 4 x 12 lanes x merged batches, gpurun_out/r6v2)
FRONT_STREAM = switches.flag("FRONT_STREAM", True)
FRONT_STREAM_MAX_LANES = 24
# Single-batch latency (one forward alone on the GPU is one dependent chain of ~50 kernels): work
# that does not depend on the chain's previous kernel runs beside it on a side stream -- the
# level-1 spatial index (input points only) beside the level-1 FPS, the level-2/3 input
# projection (the previous level's features only) beside that level's WFPS + kNN, CoarseReg's two
# kNN selections beside the grouped head products and its neighbour head beside the first
# similarity gather -- and the MLP heads take one row tile per workgroup.  On only where
# chain_fork() enables it (the 1-lane GraphPipeline and bench.py's eager latency figure): with
# many lanes in flight the chip is already full and a fork only adds streams.
CHAIN_FORK = switches.flag("CHAIN_FORK", True)
# Level-1 FPS over the spatial index's sorted copy with exact pruning (hreg_fps_indexed): the
# index is built first and the FPS skips the point groups its new centre cannot change; the same
# selections.  Clouds of FPS_SORTED_N points (fps.hip fps_sorted_kernel: points in registers) and,
# r6, 16384 < n <= 65536 with n % 64 == 0 (fps_blocks_kernel: Model_V2's 65536-point clouds on ONE
# workgroup each instead of the cluster kernel's 32 spinning single-wave participants).
FPS_SORTED = switches.flag("FPS_SORTED", True)
# the multi-lane executor's batched level-1 stage on the small-footprint pruned FPS
# (hreg_fps_indexed_lean: 4 waves x 108 VGPRs per cloud instead of 8 x 229, so the lanes' level
# kernels keep most of a CU while its cloud's FPS runs).  r6, tools/ab_graph.py paired in one
# process (gpurun_out/r6pr): 8842 vs 8624 pairs/s; the level-1 FPS served from a cache (probe)
# 9255, the whole level-1 grouping 10203.  The single-batch path keeps fps_sorted_kernel (its
# shorter iteration is the latency).
FPS_LEAN = switches.flag("FPS_LEAN", True)
FPS_SORTED_N = 16384


def fps_indexed_ok(n: int) -> bool:
    """clouds of n points that hreg_fps_indexed's pruned kernels take"""
    return n == FPS_SORTED_N or (FPS_SORTED_N < n <= 65536 and n % 64 == 0)


@dataclass
class Lin:
    W: torch.Tensor       # [N][K] contiguous f32
    alpha: torch.Tensor   # [N]
    beta: torch.Tensor    # [N]
    relu: bool = True

    @property
    def N(self):
        return self.W.shape[0]

    @property
    def K(self):
        return self.W.shape[1]


def _bn_fold(sd, pre, bias=None):
    g = sd[pre + ".weight"].float()
    b = sd[pre + ".bias"].float()
    mean = sd[pre + ".running_mean"].float()
    var = sd[pre + ".running_var"].float()
    alpha = g * (1.0 / torch.sqrt(var + BN_EPS))
    if bias is None:
        beta = b - mean * alpha
    else:
        beta = b + (bias.float() - mean) * alpha
    return alpha.contiguous(), beta.contiguous()


def _fold_bn(lin: Lin) -> Lin:
    """The bf16x6 kernels' form of a conv + eval-BN layer: alpha folded into the weight
    rows (W' = diag(alpha) W), the epilogue section [1 | beta]; the kernels start the
    accumulators from beta and apply the ReLU alone.  Same function up to fp32 rounding
    (alpha * sum w x vs sum (alpha w) x)."""
    return Lin((lin.W * lin.alpha[:, None]).contiguous(), torch.ones_like(lin.alpha),
               lin.beta.clone(), lin.relu)


def _fold_all(lins):
    return [_fold_bn(l) for l in lins]


def _conv_bn(sd, conv, bn, perm=None):
    W = sd[conv + ".weight"].float()
    W = W.reshape(W.shape[0], -1)
    if perm is not None:
        W = W[:, perm]
    bias = sd.get(conv + ".bias")
    a, b = _bn_fold(sd, bn, bias)
    return Lin(W.contiguous(), a, b, True)


def _stack(sd, pre, n, perm0=None):
    return [_conv_bn(sd, f"{pre}.{3 * i}", f"{pre}.{3 * i + 1}", perm0 if i == 0 else None)
            for i in range(n)]


def _mlp_head(sd, pre):
    """mlp1, mlp2 (Conv1d+BN+ReLU) and mlp3 (Conv1d C->1)."""
    m1 = _conv_bn(sd, pre + ".mlp1.0", pre + ".mlp1.1")
    m2 = _conv_bn(sd, pre + ".mlp2.0", pre + ".mlp2.1")
    w3 = sd[pre + ".mlp3.0.weight"].float().reshape(-1).contiguous()
    b3 = sd[pre + ".mlp3.0.bias"].float().reshape(-1).contiguous()
    return m1, m2, w3, b3


def _perm_coarse(C):
    """CoarseReg input order (layers.py:364-380) -> [geom10, w2, sims4, desc C, knn_desc C]."""
    return (list(range(10)) + [10 + 2 * C, 11 + 2 * C] + list(range(12 + 2 * C, 16 + 2 * C))
            + list(range(10, 10 + C)) + list(range(10 + C, 10 + 2 * C)))


def _perm_fine(C):
    """FineReg input order (layers.py:444-445) -> [geom10, w2, feat C, knn_feat C]."""
    return (list(range(10)) + [10 + 2 * C, 11 + 2 * C] + list(range(10, 10 + C))
            + list(range(10 + C, 10 + 2 * C)))


def _pad_coarse_convs1(sd: dict, use_sim: bool, use_neighbor: bool) -> None:
    """CoarseReg's variants (layers.py:237-244): convs_1[0] over 2C + 14 inputs (one pair of
    similarity features) or 2C + 12 (none).  In place: the weight is widened to the 2C + 16
    layout of use_sim = use_neighbor = True ([geom 10 | desc C | knn_desc C | w 2 | cos 2 |
    nbr cos 2], layers.py:368-379) with zero columns where a variant has no feature -- the
    engine then feeds zeros there, and every product of a zero column is an exact 0, so the
    fused kernels compute the variant's function."""
    key = "coarse_corres.convs_1.0.weight"
    W = sd.get(key)
    if W is None:
        return
    n = W.shape[1] - 12 - 2 * (use_sim + use_neighbor)  # 2C
    C = sd["coarse_corres.convs_2.0.weight"].shape[0] if "coarse_corres.convs_2.0.weight" in sd else n // 2
    if n != 2 * C:
        raise ValueError(f"coarse_corres.convs_1.0.weight has {W.shape[1]} inputs: not a CoarseReg over "
                         f"{C} channels with use_sim={use_sim}, use_neighbor={use_neighbor}")
    if use_sim and use_neighbor:
        return
    W16 = torch.zeros((W.shape[0], n + 16) + tuple(W.shape[2:]), dtype=W.dtype)
    W16[:, :n + 12] = W[:, :n + 12]
    o = n + 12
    if use_sim:
        W16[:, n + 12:n + 14] = W[:, o:o + 2]
        o += 2
    if use_neighbor:
        W16[:, n + 14:n + 16] = W[:, o:o + 2]
    sd[key] = W16


class PreparedWeights:
    """Device-resident folded weights for one HRegNet state dict (coarse_variant: the CoarseReg
    head's (use_sim, use_neighbor), layers.py:229-244)."""

    def __init__(self, sd: dict, device, coarse_variant=(True, True)):
        # fold on the host in fp32, then move the folded tensors to the device
        sd = {k: v.detach().to("cpu", torch.float32) if v.is_floating_point() else v
              for k, v in sd.items()}
        self.coarse_use_sim, self.coarse_use_nbr = (bool(v) for v in coarse_variant)
        _pad_coarse_convs1(sd, self.coarse_use_sim, self.coarse_use_nbr)
        fe = "feature_extraction."
        self.det, self.det_head, self.desc, self.desc_mlp = [], [], [], []
        for lvl in range(3):
            d = f"{fe}detector_{lvl + 1}"
            self.det.append(_stack(sd, d + ".convs", 3))
            self.det_head.append(_mlp_head(sd, d))
            e = f"{fe}desc_extractor_{lvl + 1}"
            self.desc.append(_stack(sd, e + ".convs", 3))
            self.desc_mlp.append([_conv_bn(sd, e + ".mlp1.0", e + ".mlp1.1"),
                                  _conv_bn(sd, e + ".mlp2.0", e + ".mlp2.1")])
        # [W_det_f; W_desc_f] of the level's two first convs (columns 4: of [geom 4 | feat])
        self.level_pre = [None] + [
            Lin(torch.cat([self.det[lv][0].W[:, 4:], self.desc[lv][0].W[:, 4:]]).contiguous(),
                torch.ones(2 * self.det[lv][0].N), torch.zeros(2 * self.det[lv][0].N), False)
            for lv in (1, 2)]
        # the same for the bf16x6 level kernels (folded BN): alpha-scaled rows and the two
        # layers' beta in the epilogue, so a precomputed row is the whole accumulator start
        self.level_pre6 = [None] + [
            Lin(torch.cat([(self.det[lv][0].W[:, 4:] * self.det[lv][0].alpha[:, None]),
                           (self.desc[lv][0].W[:, 4:] * self.desc[lv][0].alpha[:, None])]).contiguous(),
                torch.ones(2 * self.det[lv][0].N),
                torch.cat([self.det[lv][0].beta, self.desc[lv][0].beta]).contiguous(), False)
            for lv in (1, 2)]
        C = 256
        self.coarse_convs1 = _stack(sd, "coarse_corres.convs_1", 3, _perm_coarse(C))
        # convs_1[0] split by input block (COARSE_SPLIT): the 16 per-row columns, and
        # [W_desc; W_knn_desc] stacked as one batch-2 weight for the per-keypoint products
        c0 = self.coarse_convs1[0]
        self.coarse_c1_small = Lin(c0.W[:, :16].contiguous(), c0.alpha, c0.beta, True)
        self.coarse_c1_desc = Lin(torch.stack([c0.W[:, 16:16 + C], c0.W[:, 16 + C:]]).contiguous(),
                                  torch.ones(c0.N), torch.zeros(c0.N), False)
        # coarse6.hip (folded BN): alpha-scaled desc / knn_desc blocks
        self.coarse_c1_desc6 = Lin((self.coarse_c1_desc.W * c0.alpha[None, :, None]).contiguous(),
                                   torch.ones(c0.N), torch.zeros(c0.N), False)
        self.coarse_convs2 = _stack(sd, "coarse_corres.convs_2", 3)
        n0 = self.coarse_convs2[0]
        self.nbr_pre = Lin(n0.W[:, :C].contiguous(), torch.ones(n0.N), torch.zeros(n0.N), False)
        # nbr_head6_kernel (folded BN): alpha-scaled descriptor block, convs_2[0]'s beta
        self.nbr_pre6 = Lin((n0.W[:, :C] * n0.alpha[:, None]).contiguous(), torch.ones(n0.N),
                            n0.beta.clone(), False)
        self.coarse_head = _mlp_head(sd, "coarse_corres")
        self.fine = {}
        for name, C in (("fine_corres_2", 128), ("fine_corres_1", 64)):
            self.fine[name] = (_stack(sd, name + ".convs_1", 3, _perm_fine(C)), _mlp_head(sd, name))
        # [W_f; W_knn_f] of each FineReg convs_1[0] as one batch-2 weight (HEAD_PRE)
        self.fine_pre = {}
        for name, C in (("fine_corres_2", 128), ("fine_corres_1", 64)):
            f0 = self.fine[name][0][0]
            self.fine_pre[name] = Lin(torch.stack([f0.W[:, 12:12 + C], f0.W[:, 12 + C:]]).contiguous(),
                                      torch.ones(f0.N), torch.zeros(f0.N), False)
        # fine_head6_kernel (folded BN): alpha-scaled descriptor blocks (its beta is added
        # in the kernel: the batch-2 GEMM shares one epilogue)
        self.fine_pre6 = {n: Lin((l.W * self.fine[n][0][0].alpha[None, :, None]).contiguous(), l.alpha,
                                 l.beta, False) for n, l in self.fine_pre.items()}
        # Model_V2's FineReg2.mlpx (model_v2/layers.py:457-459), when the state dict has it
        self.mlpx = (_conv_bn(sd, "fine_corres_2.mlpx.0", "fine_corres_2.mlpx.1")
                     if "fine_corres_2.mlpx.0.weight" in sd else None)
        # the fp32-MFMA checker kernels' tables (libhregnet_checkers.so, test-only): built on
        # first use by a debug switch / a test, never by the product path
        det, desc, dmlp = list(self.det), list(self.desc), list(self.desc_mlp)  # (host copies)
        self._lazy = {
            "l1_table": lambda: l1_table(det[0], desc[0], dmlp[0]),
            "l2_table": lambda: l2_table(det[1], desc[1], dmlp[1]),
            "l3_table": lambda: l2_table(det[2], desc[2], dmlp[2]),
            "l2s_table": lambda: split_table(det[1], desc[1], dmlp[1]),
            "l3s_table": lambda: split_table(det[2], desc[2], dmlp[2]),
        }
        self.l1_table6 = l1_table6(_fold_all(self.det[0]), _fold_all(self.desc[0]),
                                   _fold_all(self.desc_mlp[0]))
        self.l2_table6 = l2_table6(*(_fold_all(x) for x in (self.det[1], self.desc[1], self.desc_mlp[1])))
        self.l3_table6 = l2_table6(*(_fold_all(x) for x in (self.det[2], self.desc[2], self.desc_mlp[2])))
        self.l2s_table6 = split_table6(*(_fold_all(x) for x in (self.det[1], self.desc[1], self.desc_mlp[1])))
        self.l3s_table6 = split_table6(*(_fold_all(x) for x in (self.det[2], self.desc[2], self.desc_mlp[2])))
        self.fine_table = {name: fine_head_table(self.fine[name][0], C)
                           for name, C in (("fine_corres_2", 128), ("fine_corres_1", 64))}
        self.nbr_table = nbr_head_table(self.coarse_convs2, 256)
        self.fine_table6 = {name: fine_head_table6(_fold_all(self.fine[name][0]))
                            for name in ("fine_corres_2", "fine_corres_1")}
        self.nbr_table6 = nbr_head_table6(_fold_all(self.coarse_convs2), 256)
        self.coarse_table6 = coarse_head_table6(_fold_bn(self.coarse_c1_small),
                                                _fold_all(self.coarse_convs1))
        self.head_table = {("det", lvl): mlp_head_table(self.det_head[lvl]) for lvl in range(3)}
        self.head_table["coarse"] = mlp_head_table(self.coarse_head)
        for name in ("fine_corres_2", "fine_corres_1"):
            self.head_table[name] = mlp_head_table(self.fine[name][1])
        self.head_table6 = {k: mlp_head_table6(h) for k, h in (
            [(("det", lvl), self.det_head[lvl]) for lvl in range(3)] + [("coarse", self.coarse_head)] +
            [(n, self.fine[n][1]) for n in ("fine_corres_2", "fine_corres_1")])}
        for attr in ("det", "det_head", "desc", "desc_mlp", "coarse_convs1", "coarse_c1_small",
                     "coarse_c1_desc", "coarse_convs2", "nbr_pre", "fine_pre", "fine_pre6", "nbr_pre6", "level_pre", "level_pre6", "coarse_c1_desc6",
                     "coarse_head", "fine", "l1_table6", "l2_table6",
                     "l3_table6", "l2s_table6", "l3s_table6",
                     "fine_table", "fine_table6", "nbr_table6", "coarse_table6",
                     "nbr_table", "head_table", "head_table6", "mlpx"):
            setattr(self, attr, _to_device(getattr(self, attr), device))
        self._device = device

    def __getattr__(self, name):
        lazy = self.__dict__.get("_lazy")
        if lazy is None or name not in lazy:
            raise AttributeError(name)
        t = _to_device(lazy.pop(name)(), self.__dict__["_device"])
        setattr(self, name, t)
        return t


# ---------------------------------------------------------- fused level 1
def frag_layer(W: torch.Tensor) -> torch.Tensor:
    """MFMA A-fragments of a layer W [Cout][Cin] (Cin, Cout multiples of 32) for the
    accumulator-chaining order of group_l1.hip: [co][ct][q][lane] =
    W[co*32 + (lane & 31)][ct*32 + (q & 3) + 8*(q >> 2) + 4*(lane >> 5)]."""
    Cout, Cin = W.shape
    co = torch.arange(Cout // 32).view(-1, 1, 1, 1)
    ct = torch.arange(Cin // 32).view(1, -1, 1, 1)
    q = torch.arange(16).view(1, 1, -1, 1)
    lane = torch.arange(64).view(1, 1, 1, -1)
    rows = co * 32 + (lane & 31)
    cols = ct * 32 + (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5)
    return W[rows, cols].reshape(-1)


def frag_geom(W: torch.Tensor) -> torch.Tensor:
    """First layer (Cin = 4): k-step s, lane half h takes channel 2h + s -> [s][lane]."""
    s = torch.arange(2).view(-1, 1)
    lane = torch.arange(64).view(1, -1)
    return W[lane & 31, 2 * (lane >> 5) + s].reshape(-1)


def frag_input(W: torch.Tensor) -> torch.Tensor:
    """First layer over [geom 4 | feature CF] (group_l2.hip conv_in): geom k-step s, lane
    half h -> channel 2h + s, [co][s][lane]; feature k-step s, half h -> channel
    4 + h*CF/2 + s, [co][s][lane].  Returns (geom fragments, feature fragments)."""
    Cout, K = W.shape
    TF = (K - 4) // 2
    co = torch.arange(Cout // 32).view(-1, 1, 1)
    lane = torch.arange(64).view(1, 1, -1)
    rows = co * 32 + (lane & 31)
    sg = torch.arange(2).view(1, -1, 1)
    geom = W[rows, 2 * (lane >> 5) + sg]
    sf = torch.arange(TF).view(1, -1, 1)
    feat = W[rows, 4 + (lane >> 5) * TF + sf]
    return geom.reshape(-1), feat.reshape(-1)


def _win(cout_tiles: int, nstep: int) -> int:
    """k-steps per prefetch window of a group_fused.hip call (first_win / win_for)."""
    w = 2 if cout_tiles >= 8 else 4 if cout_tiles >= 4 else 8
    return min(w, nstep)


def _grouped(frag: torch.Tensor, cout_tiles: int, nstep: int) -> torch.Tensor:
    """[co][step][lane] fragments -> [co][step group][lane][GS]: GS = min(4, window)
    consecutive k-steps innermost per lane, so the kernel fetches them with one
    global_load_dwordx4 (x2)."""
    gs = min(4, _win(cout_tiles, nstep))
    f = frag.reshape(cout_tiles, nstep // gs, gs, 64)
    return f.transpose(-1, -2).reshape(-1)


def frag_segment(W: torch.Tensor, col0: int, width: int) -> torch.Tensor:
    """A fragments of input columns [col0, col0 + width) streamed as B from a row:
    k-step s, lane half h -> column col0 + h*width/2 + s; [co][width/2][lane]."""
    Cout = W.shape[0]
    co = torch.arange(Cout // 32).view(-1, 1, 1)
    lane = torch.arange(64).view(1, 1, -1)
    s = torch.arange(width // 2).view(1, -1, 1)
    return W[co * 32 + (lane & 31), col0 + (lane >> 5) * (width // 2) + s].reshape(-1)


def fine_head_table(convs, C: int) -> torch.Tensor:
    """Weight/epilogue table of group_head.hip's FineReg kernel: convs_1 with the input
    columns in the packed order [small 12, pad 4, f_src C, f_dst C] (_perm_fine + 4 zero
    columns), fragments grouped like l2_table."""
    W1 = convs[0].W
    N1 = W1.shape[0]
    T1 = N1 // 32
    W1p = torch.cat([W1[:, :12], torch.zeros(N1, 4, dtype=W1.dtype), W1[:, 12:]], 1)
    parts = [_grouped(frag_segment(W1p, 0, 16), T1, 8),
             _grouped(frag_segment(W1p, 16, C), T1, C // 2),
             _grouped(frag_segment(W1p, 16 + C, C), T1, C // 2),
             _grouped(frag_layer(convs[1].W), T1, T1 * 16),
             _grouped(frag_layer(convs[2].W), T1, T1 * 16)]
    for lin in convs:
        parts += [lin.alpha, lin.beta]
    return torch.cat([p.reshape(-1).float() for p in parts]).contiguous()


def nbr_head_table(convs, C: int) -> torch.Tensor:
    """Table of group_head.hip's CoarseReg neighbour-branch kernel: convs_2 over the
    columns [desc C | geom 4] (the order engine.coarse_reg assembles)."""
    T1 = convs[0].W.shape[0] // 32
    W1 = convs[0].W
    parts = [_grouped(frag_segment(W1, 0, C), T1, C // 2), _grouped(frag_segment(W1, C, 4), T1, 2),
             _grouped(frag_layer(convs[1].W), T1, T1 * 16),
             _grouped(frag_layer(convs[2].W), T1, T1 * 16)]
    for lin in convs:
        parts += [lin.alpha, lin.beta]
    return torch.cat([p.reshape(-1).float() for p in parts]).contiguous()


def _head_table6(first, T1: int, nfirst: int, convs) -> torch.Tensor:
    """Table of group_head.hip's bf16x6 head kernels (Head6Cfg): the narrow first block
    (nfirst f32 k-steps, zero-padded to one chunk), conv 2, conv 3 as bf16 piece chunk
    fragments (frag6), then the three f32 epilogues."""
    parts = [frag6(first, T1, nfirst), frag6(frag_layer(convs[1].W), T1, T1 * 16),
             frag6(frag_layer(convs[2].W), T1, T1 * 16)]
    for lin in convs:
        parts += [lin.alpha, lin.beta]
    return torch.cat([p.reshape(-1).float() for p in parts]).contiguous()


def coarse_head_table6(small: Lin, convs) -> torch.Tensor:
    """Table of coarse6.hip: convs_1[0]'s 16 small columns (frag_segment: k-step s of lane
    half h <-> column 8h + s, one chunk), convs_1[1], convs_1[2] as bf16 piece chunk
    fragments, then alpha/beta of the three layers (convs_1[0]'s from the split Lin)."""
    T = small.W.shape[0] // 32
    parts = [frag6(frag_segment(small.W, 0, 16), T, 8), frag6(frag_layer(convs[1].W), T, T * 16),
             frag6(frag_layer(convs[2].W), T, T * 16)]
    for lin in (small, convs[1], convs[2]):
        parts += [lin.alpha, lin.beta]
    return torch.cat([p.reshape(-1).float() for p in parts]).contiguous()


def fine_head_table6(convs) -> torch.Tensor:
    """FineReg convs_1 for fine_head6_kernel: the 16 small columns [small 12, pad 4] of
    convs_1[0] (its descriptor blocks are precomputed per point, HEAD_PRE)."""
    W1 = convs[0].W
    N1 = W1.shape[0]
    W1p = torch.cat([W1[:, :12], torch.zeros(N1, 4, dtype=W1.dtype)], 1)
    return _head_table6(frag_segment(W1p, 0, 16), N1 // 32, 8, convs)


def nbr_head_table6(convs, C: int) -> torch.Tensor:
    """CoarseReg convs_2 for nbr_head6_kernel: the 4 geometry columns of convs_2[0] (its
    descriptor block is precomputed per point, HEAD_PRE)."""
    W1 = convs[0].W
    return _head_table6(frag_segment(W1, C, 4), W1.shape[0] // 32, 2, convs)


def mlp_head_table(head) -> torch.Tensor:
    """Table of mlp_head.hip (HCfg): mlp1 and mlp2 fragments (frag_layer, 4 k-steps
    innermost per lane), alpha1, beta1, alpha2, beta2, w3, b3 (+3 pad)."""
    m1, m2, w3, b3 = head
    parts = [_group4(frag_layer(m1.W), 4), _group4(frag_layer(m2.W), 4), m1.alpha, m1.beta,
             m2.alpha, m2.beta, w3, b3, torch.zeros(3)]
    return torch.cat([p.reshape(-1).float() for p in parts]).contiguous()


def mlp_head_table6(head) -> torch.Tensor:
    """Table of hreg_mlp_head6 (HCfg TABLE6): mlp1 and mlp2 (folded BN, _fold_bn) as bf16
    piece chunk fragments (frag6), then mlp_head_table's epilogue section."""
    m1, m2, w3, b3 = head
    m1, m2 = _fold_bn(m1), _fold_bn(m2)
    T = m1.W.shape[0] // 32
    parts = [frag6(frag_layer(m1.W), T, T * 16), frag6(frag_layer(m2.W), T, T * 16), m1.alpha,
             m1.beta, m2.alpha, m2.beta, w3, b3, torch.zeros(3)]
    return torch.cat([p.reshape(-1).float() for p in parts]).contiguous()


def l2_table(det, desc, mlp) -> torch.Tensor:
    """Weight/epilogue table of the fused level-2/3 kernel (layout: group_fused.hip Cfg)."""
    T1, T3 = det[0].W.shape[0] // 32, det[2].W.shape[0] // 32
    TM1, TM2 = mlp[0].W.shape[0] // 32, mlp[1].W.shape[0] // 32
    TF = (det[0].W.shape[1] - 4) // 2
    parts = []
    for stack in (det, desc):
        g, f = frag_input(stack[0].W)
        parts += [_grouped(g, T1, 2), _grouped(f, T1, TF),
                  _grouped(frag_layer(stack[1].W), T1, T1 * 16),
                  _grouped(frag_layer(stack[2].W), T3, T1 * 16)]
    parts += [_grouped(frag_layer(mlp[0].W), TM1, 3 * T3 * 16),
              _grouped(frag_layer(mlp[1].W), TM2, TM1 * 16)]
    for lin in (det[0], det[1], det[2], desc[0], desc[1], desc[2], mlp[0], mlp[1]):
        parts += [lin.alpha, lin.beta]
    return torch.cat([p.reshape(-1).float() for p in parts]).contiguous()


def _bf16_pieces(x: torch.Tensor) -> torch.Tensor:
    """Exact truncation split of fp32 x into hi + mid + lo bf16 values (mfma_chain.h
    split8): -> int16 bit patterns [3, *x.shape]."""
    x = x.float().contiguous()
    mask = torch.tensor(-65536, dtype=torch.int32)  # 0xffff0000
    xb = x.view(torch.int32)
    r = x - (xb & mask).view(torch.float32)
    rb = r.view(torch.int32)
    lo = r - (rb & mask).view(torch.float32)
    out = []
    for v in (xb, rb, lo.view(torch.int32)):
        u = (v >> 16) & 0xFFFF
        out.append(torch.where(u >= 32768, u - 65536, u).to(torch.int16))
    return torch.stack(out)


def frag6(frag: torch.Tensor, cout_tiles: int, nstep: int) -> torch.Tensor:
    """f32 A-fragments [co][k-step][lane] (nstep k-steps, zero-padded to a multiple of 8)
    -> the bf16x6 table block [co][chunk][piece][lane][8] (as float32 words): chunk c of
    a lane holds its f32 fragments of k-steps 8c .. 8c+7 (mfma_chain.h, bf16x6)."""
    f = frag.reshape(cout_tiles, nstep, 64).float()
    pad = (-nstep) % 8
    if pad:
        f = torch.cat([f, torch.zeros(cout_tiles, pad, 64)], 1)
    nch = f.shape[1] // 8
    f = f.reshape(cout_tiles, nch, 8, 64).transpose(2, 3)      # [co][chunk][lane][8]
    p = _bf16_pieces(f).permute(1, 2, 0, 3, 4).contiguous()   # [co][chunk][piece][lane][8]
    return p.view(torch.float32).reshape(-1)


def l2_table6(det, desc, mlp) -> torch.Tensor:
    """Table of group_fused6.hip (Cfg6): bf16x6 chunk fragments of every layer in
    l2_table's block order (the 2-step geometry block zero-padded to one chunk), then the
    f32 epilogues."""
    T1, T3 = det[0].W.shape[0] // 32, det[2].W.shape[0] // 32
    TM1, TM2 = mlp[0].W.shape[0] // 32, mlp[1].W.shape[0] // 32
    TF = (det[0].W.shape[1] - 4) // 2
    parts = []
    for stack in (det, desc):
        g, f = frag_input(stack[0].W)
        parts += [frag6(g, T1, 2), frag6(f, T1, TF), frag6(frag_layer(stack[1].W), T1, T1 * 16),
                  frag6(frag_layer(stack[2].W), T3, T1 * 16)]
    parts += [frag6(frag_layer(mlp[0].W), TM1, 3 * T3 * 16),
              frag6(frag_layer(mlp[1].W), TM2, TM1 * 16)]
    for lin in (det[0], det[1], det[2], desc[0], desc[1], desc[2], mlp[0], mlp[1]):
        parts += [lin.alpha, lin.beta]
    return torch.cat([p.reshape(-1).float() for p in parts]).contiguous()


def split_table(det, desc, mlp) -> torch.Tensor:
    """Weight/epilogue table of group_split.hip: the l2_table blocks and epilogues, with
    every block grouped 4 k-steps innermost per lane (the 2-step geometry block: 2)."""
    parts = []
    for stack in (det, desc):
        g, f = frag_input(stack[0].W)
        parts += [_group4(g, 2), _group4(f, 4), _group4(frag_layer(stack[1].W), 4),
                  _group4(frag_layer(stack[2].W), 4)]
    parts += [_group4(frag_layer(mlp[0].W), 4), _group4(frag_layer(mlp[1].W), 4)]
    # mlp1's x2 block row-major [CM1][C3] (group_split.hip: per-group matrix-vector product)
    parts += [mlp[0].W[:, :det[2].W.shape[0]].contiguous()]
    for lin in (det[0], det[1], det[2], desc[0], desc[1], desc[2], mlp[0], mlp[1]):
        parts += [lin.alpha, lin.beta]
    return torch.cat([p.reshape(-1).float() for p in parts]).contiguous()


def split_table6(det, desc, mlp) -> torch.Tensor:
    """Table of group_split6.hip (SCfg6): l2_table6's bf16 piece chunk fragments, then
    mlp1's x2 block f32 row-major [CM1][C3] (the per-group matrix-vector product), then the
    f32 epilogues."""
    t6 = l2_table6(det, desc, mlp)
    ne = sum(2 * lin.N for lin in (det[0], det[1], det[2], desc[0], desc[1], desc[2], mlp[0], mlp[1]))
    x2 = mlp[0].W[:, :det[2].W.shape[0]].contiguous().reshape(-1).float()
    return torch.cat([t6[:t6.numel() - ne], x2, t6[t6.numel() - ne:]]).contiguous()


def _group4(frag: torch.Tensor, gs: int) -> torch.Tensor:
    """[blocks][steps][lane] -> [blocks][steps/gs][lane][gs] (gs k-steps innermost)."""
    f = frag.reshape(-1, gs, 64)
    return f.transpose(-1, -2).reshape(-1)


def l1_table(det, desc, mlp) -> torch.Tensor:
    """Weight/epilogue table of the fused level-1 kernel (layout: group_l1.hip F_*/E_*;
    fragments with 2 (first layer) or 4 consecutive k-steps innermost per lane)."""
    parts = [_group4(frag_geom(det[0].W), 2), _group4(frag_layer(det[1].W), 4),
             _group4(frag_layer(det[2].W), 4),
             _group4(frag_geom(desc[0].W), 2), _group4(frag_layer(desc[1].W), 4),
             _group4(frag_layer(desc[2].W), 4),
             _group4(frag_layer(mlp[0].W), 4), _group4(frag_layer(mlp[1].W), 4)]
    for lin in (det[0], det[1], det[2], desc[0], desc[1], desc[2], mlp[0], mlp[1]):
        parts += [lin.alpha, lin.beta]
    return torch.cat([p.reshape(-1).float() for p in parts]).contiguous()


def l1_table6(det, desc, mlp) -> torch.Tensor:
    """Table of group_l1_6.hip: l1_table's blocks as bf16 piece chunk fragments (frag6;
    the 2-step geometry blocks zero-padded to one chunk), then the same f32 epilogues."""
    parts = [frag6(frag_geom(det[0].W), 1, 2), frag6(frag_layer(det[1].W), 1, 16),
             frag6(frag_layer(det[2].W), 2, 16),
             frag6(frag_geom(desc[0].W), 1, 2), frag6(frag_layer(desc[1].W), 1, 16),
             frag6(frag_layer(desc[2].W), 2, 16),
             frag6(frag_layer(mlp[0].W), 1, 96), frag6(frag_layer(mlp[1].W), 2, 16)]
    for lin in (det[0], det[1], det[2], desc[0], desc[1], desc[2], mlp[0], mlp[1]):
        parts += [lin.alpha, lin.beta]
    return torch.cat([p.reshape(-1).float() for p in parts]).contiguous()


def _to_device(x, device):
    if isinstance(x, torch.Tensor):
        return x.to(device).contiguous()
    if isinstance(x, Lin):
        return Lin(_to_device(x.W, device), _to_device(x.alpha, device),
                   _to_device(x.beta, device), x.relu)
    if isinstance(x, (list, tuple)):
        return type(x)(_to_device(v, device) for v in x)
    if isinstance(x, dict):
        return {k: _to_device(v, device) for k, v in x.items()}
    return x


# ---------------------------------------------------------------- launchers

def _seg(base, k0, kc, ld=None, gather=None, rowscale=None, row_div=1, batch_stride=0):
    s = Seg()
    s.base = base.data_ptr()
    s.gather = gather.data_ptr() if gather is not None else None
    s.rowscale = rowscale.data_ptr() if rowscale is not None else None
    s.batch_stride = batch_stride
    s.ld = base.shape[-1] if ld is None else ld
    s.k0, s.kc, s.row_div = k0, kc, row_div
    return s


def gemm(segs, lin: Lin, R: int, out: torch.Tensor | None = None, adds=(), b6=False):
    """out[R][N] = act(alpha * (A @ W^T + sum(adds)) + beta), A assembled from segs;
    adds: up to 2 row sources (_seg with row_div or gather) of [*, N] addends;
    b6: on hreg_gemm6 (bf16x6 products) when B6_GEMM (no addends)."""
    if out is None:
        out = torch.empty((R, lin.N), device=lin.W.device, dtype=torch.float32)
    g = _gemm_struct(segs, lin, R, out, adds)
    if b6 and B6_GEMM and not adds:
        _lib.gemm6(g)
    else:
        _lib.gemm(g)
    return out


def _gemm_struct(segs, lin: Lin, R: int, out: torch.Tensor, adds=()) -> Gemm:
    """the hreg_gemm_t of gemm() (not launched)"""
    g = Gemm()
    for i, s in enumerate(segs):
        g.seg[i] = s
    g.nseg = len(segs)
    for i, s in enumerate(adds):
        g.add[i] = s
    g.nadd = len(adds)
    g.R, g.N, g.K = R, lin.N, lin.K
    g.batch = 1
    g.ldw = lin.K
    g.w_batch_stride = 0
    g.W = lin.W.data_ptr()
    g.scale = lin.alpha.data_ptr()
    g.shift = lin.beta.data_ptr()
    g.relu = 1 if lin.relu else 0
    g.epi = _lib.HREG_EPI_AFFINE
    g.out = out.data_ptr()
    g.ldo = out.shape[-1]
    g.out_batch_stride = 0
    return g


def _gemm_batched_desc(lin: Lin, desc3, rows: int, C: int, out, x1=None):
    """out[i] = x_i @ lin.W[i]^T for i in {0, 1}, x_0 = desc3[:rows], x_1 = desc3[rows:2 rows]
    (or x1 when given and not contiguous after x_0: then two launches); one launch with
    grid.z = 2 otherwise; lin.W [2][N][C], identity epilogue."""
    if x1 is not None and x1.data_ptr() != desc3.data_ptr() + rows * C * 4:
        for i, x in enumerate((desc3, x1)):
            gemm([_seg(x, 0, C, ld=C)], Lin(lin.W[i], lin.alpha, lin.beta, False), rows, out=out[i])
        return out
    _lib.gemm(_batched_desc_struct(lin, desc3, rows, C, out))
    return out


def _batched_desc_struct(lin: Lin, desc3, rows: int, C: int, out) -> Gemm:
    """the batch-2 hreg_gemm_t of _gemm_batched_desc (x_1 contiguous after x_0; not launched)"""
    N = lin.W.shape[1]
    g = Gemm()
    g.seg[0] = _seg(desc3, 0, C, ld=C, batch_stride=rows * C)
    g.nseg = 1
    g.R, g.N, g.K = rows, N, C
    g.batch = 2
    g.ldw = C
    g.w_batch_stride = N * C
    g.W = lin.W.data_ptr()
    g.scale = lin.alpha.data_ptr()
    g.shift = lin.beta.data_ptr()
    g.relu = 0
    g.epi = _lib.HREG_EPI_AFFINE
    g.out = out.data_ptr()
    g.ldo = N
    g.out_batch_stride = rows * N
    return g


def cosine_gemm(a, b, na, nb_, nb: int, n1: int, n2: int, C: int, out):
    """S[b][i][j] = <a_i, b_j> / (|a_i||b_j| + 1e-6) per pair (layers.py:29-41)."""
    _lib.gemm(_cosine_struct(a, b, na, nb_, nb, n1, n2, C, out))
    return out


def _cosine_struct(a, b, na, nb_, nb: int, n1: int, n2: int, C: int, out) -> Gemm:
    g = Gemm()
    g.seg[0] = _seg(a, 0, C, ld=C, batch_stride=n1 * C)
    g.nseg = 1
    g.R, g.N, g.K = n1, n2, C
    g.batch = nb
    g.ldw = C
    g.w_batch_stride = n2 * C
    g.W = b.data_ptr()
    g.relu = 0
    g.epi = _lib.HREG_EPI_COSINE
    g.rnorm = na.data_ptr()
    g.cnorm = nb_.data_ptr()
    g.rnorm_batch_stride = n1
    g.cnorm_batch_stride = n2
    g.out = out.data_ptr()
    g.ldo = n2
    g.out_batch_stride = n1 * n2
    return g


def _stream():
    return _lib.stream_handle()


def _empty(*shape, dtype=torch.float32, device):
    return torch.empty(shape, dtype=dtype, device=device)


_fork_on = False
_fork_side = None
_fork_streams = {}


class chain_fork:
    """Context: enable the single-forward side-stream forks (CHAIN_FORK) inside it, on `side`
    (a stream the caller owns: required for forks inside a graph capture, where no stream is
    created) or else on a stream made per forking stream."""

    def __init__(self, side=None):
        self.side = side

    def __enter__(self):
        global _fork_on, _fork_side
        self.prev = (_fork_on, _fork_side)
        _fork_on, _fork_side = CHAIN_FORK, self.side
        return self

    def __exit__(self, *exc):
        global _fork_on, _fork_side
        _fork_on, _fork_side = self.prev
        return False


def _fork_begin():
    """-> (main, side) with side ordered after everything enqueued on main so far, or None
    (no fork: the work stays on main) inside a capture when main is not the capture's origin
    (HIP capture takes one level of fork/join, capture.py) or no side stream was given."""
    main = torch.cuda.current_stream()
    origin = capture.capture_origin()
    if origin is not None and main != origin:
        return None
    side = _fork_side
    if side is None:
        if origin is not None:
            return None
        side = _fork_streams.get(main.cuda_stream)
        if side is None:
            side = _fork_streams[main.cuda_stream] = torch.cuda.Stream(device=main.device)
    side.wait_stream(main)
    return main, side


# set when a multi-workgroup FPS (n > 16384) has been enqueued since the last
# check_device_status(): only those kernels raise device status bits
_status_pending = False


def check_device_status(force: bool = False):
    """Raise if a kernel flagged an error on the device since the last check (the
    multi-workgroup FPS poll timeout, HREG_STATUS_FPS_TIMEOUT: its cloud's indices were
    replaced by zeros).  Synchronous; called at the sync points the executors already
    have (GraphPipeline.run, Pipeline.run, models.*.forward when such an FPS ran)."""
    global _status_pending
    if not (_status_pending or force):
        return
    _status_pending = False
    st = _lib.device_status(clear=True)
    if st & _lib.HREG_STATUS_FPS_TIMEOUT:
        raise RuntimeError("multi-workgroup FPS: exchange poll timed out on the device; "
                           "the affected clouds' FPS indices are invalid (zeros)")
    if st:
        raise RuntimeError(f"device status {st:#x}")


def fps(xyz, npoint, weights=None, out=None, concurrent=0):
    """FPS / WFPS of nb clouds; concurrent >= 1: the caller guarantees at most that many
    multi-workgroup FPS launches run at once (hreg_fps_bounded: a larger spin budget)."""
    global _status_pending
    nb, n, _ = xyz.shape
    dev = xyz.device
    if out is None:
        idx = _empty(nb, npoint, dtype=torch.int32, device=dev)
        sampled = _empty(nb, npoint, 3, device=dev)
    else:
        idx, sampled = out
    # temp: the register kernels read a caller's temp as the initial running minima (the
    # reference's semantics), so they get none (1e10); above their sizes (n > 16384, weighted
    # n > 8192) the multi-workgroup kernel keeps its exchange slots there, or the memory kernel its
    # running minima (then from 1e10, models/utils.py:25)
    big = n > 16384 or (weights is not None and n > 8192)
    temp = torch.full((nb, n), 1e10, device=dev) if big else None
    _status_pending |= n > 16384 or (weights is not None and n > 8192)
    if weights is None and concurrent > 0:
        call("hreg_fps_bounded", nb, n, npoint, xyz, temp, idx, sampled, concurrent, _stream())
    elif weights is None:
        call("hreg_furthest_point_sampling", nb, n, npoint, xyz, temp, idx, sampled, _stream())
    else:
        call("hreg_weighted_furthest_point_sampling", nb, n, npoint, xyz, weights, temp, idx,
             sampled, _stream())
    return idx, sampled


def fps_indexed(xyz, npoint, ws, out=None, lean=False):
    """FPS of nb clouds (fps_indexed_ok sizes) over their spatial index in ws (hreg_spatial_index
    already enqueued): hreg_fps_indexed, bitwise fps(xyz, npoint).  lean: 16384-point clouds on
    the small-footprint kernel (hreg_fps_indexed_lean; the throughput executor's batched stage)."""
    nb, n, _ = xyz.shape
    if out is None:
        idx = _empty(nb, npoint, dtype=torch.int32, device=xyz.device)
        sampled = _empty(nb, npoint, 3, device=xyz.device)
    else:
        idx, sampled = out
    call("hreg_fps_indexed_lean" if lean else "hreg_fps_indexed", nb, n, npoint, xyz, ws, None, idx, sampled,
         _stream())
    return idx, sampled


def head_out(x, C, nclouds, rows, w3, b3, mode, want_weights=False):
    dev = x.device
    out = _empty(nclouds * rows, device=dev)
    wout = _empty(nclouds * rows, device=dev) if want_weights else None
    call("hreg_head_out", x, C, x.shape[-1], nclouds, rows, w3, b3, mode, out, wout, _stream())
    return out, wout


def attend(logits, G, k, vals=None, vgather=None, xyz_rows=None, want_attw=False):
    dev = logits.device
    C = logits.shape[-1]
    attw = _empty(G * k, device=dev) if want_attw else None
    att = None
    Cv = 0
    if vals is not None:
        Cv = vals.shape[-1]
        att = _empty(G, Cv, device=dev)
    kp = _empty(G, 3, device=dev) if xyz_rows is not None else None
    call("hreg_attend", logits, C, C, G, k, attw, vals, vgather, Cv, Cv, att, Cv, xyz_rows, kp,
         _stream())
    return attw, att, kp


def group_max(x, G, k):
    C = x.shape[-1]
    out = _empty(G, C, device=x.device)
    call("hreg_group_max", x, G, k, C, C, out, C, _stream())
    return out


def row_norms(x):
    out = _empty(x.shape[0], device=x.device)
    call("hreg_row_norms", x, x.shape[0], x.shape[1], x.shape[1], out, _stream())
    return out


def knn_group(q, p, k, out=None):
    """q [nb,m,3], p [nb,n,3] -> gidx [nb*m*k] int32 (global rows of p), geom [nb*m*k,4], knn_xyz."""
    nb, m, _ = q.shape
    n = p.shape[1]
    dev = q.device
    R = nb * m * k
    if out is None:
        gidx = _empty(R, dtype=torch.int32, device=dev)
        geom = _empty(R, 4, device=dev)
        kx = _empty(R, 3, device=dev)
    else:
        gidx, geom, kx = out
    call("hreg_knn_group", q, p, nb, m, n, k, gidx, geom, kx, _stream())
    return gidx, geom, kx


def spatial_index_bytes(nb: int, n: int) -> int:
    return _lib.load(require_gpu=False).hreg_spatial_index_bytes(nb, n)


def knn_group_indexed(q, p, k, ws, out=None, build=True):
    """knn_group through a per-cloud Morton spatial index built into ws (n <= 65536):
    bit-identical to knn_group, visiting only the point blocks that can hold a neighbour."""
    nb, m, _ = q.shape
    n = p.shape[1]
    dev = q.device
    R = nb * m * k
    if out is None:
        gidx = _empty(R, dtype=torch.int32, device=dev)
        geom = _empty(R, 4, device=dev)
        kx = _empty(R, 3, device=dev)
    else:
        gidx, geom, kx = out
    if build:
        call("hreg_spatial_index", p, nb, n, ws, _stream())
    call("hreg_knn_group_indexed", q, p, ws, nb, m, n, k, gidx, geom, kx, _stream())
    return gidx, geom, kx


def knn_idx32(p1, p2, k, out=None):
    b, n1, d = p1.shape
    n2 = p2.shape[1]
    idx = _empty(b, n1, k, dtype=torch.int32, device=p1.device) if out is None else out
    call("hreg_knn_points", p1, p2, b, n1, n2, d, k, None, None, idx, None, _stream())
    return idx


# ------------------------------------------------------------------ stages

SPATIAL_KNN_MIN = 4096  # clouds at least this large group through the spatial index
SPATIAL_KNN_MAX = 65536  # = csrc/knn.hip SI_MAXN


# Tests set this to a dict to receive every kNN selection of an eager forward as cloud-
# local int64 [clouds, queries, k] tensors: "knn_1".."knn_3" (src and dst clouds stacked),
# "coarse_desc_knn", "coarse_nbr" (src and dst stacked), "fine_corres_2_knn",
# "fine_corres_1_knn".  None (the default) records nothing.
INDEX_RECORD = None


def _record_knn(name, idx, nclouds, n_db, k, global_rows):
    if INDEX_RECORD is None:
        return
    i = idx.view(nclouds, -1, k).long()
    if global_rows:
        i = i - (torch.arange(nclouds, device=i.device) * n_db).view(-1, 1, 1)
    INDEX_RECORD[name] = i.clone()


def random_samples(parts: int, clouds_per_part: int, lvl_sizes, device):
    """use_fps=False (layers.py:144-147): every level draws torch.randperm(N)[:nsample] on
    the host generator, ONE draw for the whole batch of a cloud set, in the reference's
    call order (src levels 1-3, then dst levels 1-3: models.py:79-80, 26-58).  -> per level
    the local indices [parts * clouds_per_part, M] int32 on the device (each part's rows
    share its draw)."""
    draws = [[torch.randperm(n)[:LEVELS[lvl][0]] for lvl, n in enumerate(lvl_sizes)]
             for _ in range(parts)]  # part-major: the reference's call order
    out = []
    for lvl in range(len(lvl_sizes)):
        rows = [d[lvl].to(torch.int32).expand(clouds_per_part, -1) for d in draws]
        out.append(torch.cat(rows, 0).contiguous().to(device, non_blocking=False))
    return out


def random_sample_level(lvl: int, n: int, clouds: int, device):
    """one level's draw (layers.py:146) for `clouds` clouds -> [clouds, M] int32"""
    return torch.randperm(n)[:LEVELS[lvl][0]].to(torch.int32).expand(clouds, -1).contiguous().to(device)


def gather_xyz(xyz, idx):
    """xyz [nb,n,3], local idx [nb,m] int32 -> xyz[c, idx[c]] [nb,m,3] (hreg_index_offset +
    hreg_gather_rows)"""
    nb, n, _ = xyz.shape
    m = idx.shape[1]
    g = _empty(nb * m, dtype=torch.int32, device=xyz.device)
    call("hreg_index_offset", idx, nb, m, n, g, _stream())
    out = _empty(nb, m, 3, device=xyz.device)
    call("hreg_gather_rows", xyz, 3, g, nb * m, 3, out, 3, _stream())
    return out


def grouping(xyz, lvl: int, weights=None, out=None, ws=None, sample=None, fps_concurrent=0, fps_lean=False):
    """FPS/WFPS + knn_group of one level (layers.py:136-149): (idx, sampled, gidx, geom, knn_xyz).
    out: optional preallocated tensors of the same tuple; ws: spatial-index workspace
    (uint8, spatial_index_bytes) for large clouds; sample: the level's random-sampling
    indices instead of FPS (use_fps=False, random_samples).  Under chain_fork() the spatial
    index is built on a side stream while the FPS runs."""
    M, k = LEVELS[lvl][:2]
    nb, n, _ = xyz.shape
    use_si = SPATIAL_KNN_MIN <= n <= SPATIAL_KNN_MAX
    if FPS_SORTED and use_si and fps_indexed_ok(n) and weights is None and sample is None:
        # the index first: the FPS reads its Morton-sorted copy (fps_indexed), the kNN its blocks
        if ws is None:
            ws = _empty(spatial_index_bytes(nb, n), dtype=torch.uint8, device=xyz.device)
        call("hreg_spatial_index", xyz, nb, n, ws, _stream())
        idx, sampled = fps_indexed(xyz, M, ws, out=None if out is None else out[:2], lean=fps_lean)
        gidx, geom, kx = knn_group_indexed(sampled, xyz, k, ws, out=None if out is None else out[2:5],
                                           build=False)
        _record_knn(f"knn_{lvl + 1}", gidx, nb, n, k, True)
        return idx, sampled, gidx, geom, kx
    fk = _fork_begin() if (_fork_on and use_si and sample is None) else None
    if fk is not None:
        if ws is None:
            ws = _empty(spatial_index_bytes(nb, n), dtype=torch.uint8, device=xyz.device)
        main, side = fk
        with torch.cuda.stream(side):
            call("hreg_spatial_index", xyz, nb, n, ws, _stream())
        idx, sampled = fps(xyz, M, None if weights is None else weights.view(nb, n),
                           out=None if out is None else out[:2], concurrent=fps_concurrent)
        main.wait_stream(side)
        gidx, geom, kx = knn_group_indexed(sampled, xyz, k, ws, out=None if out is None else out[2:5],
                                           build=False)
        _record_knn(f"knn_{lvl + 1}", gidx, nb, n, k, True)
        return idx, sampled, gidx, geom, kx
    if sample is not None:
        idx, sampled = sample, gather_xyz(xyz, sample)
    else:
        idx, sampled = fps(xyz, M, None if weights is None else weights.view(nb, n),
                           out=None if out is None else out[:2], concurrent=fps_concurrent)
    kout = None if out is None else out[2:5]
    if use_si:
        if ws is None:
            ws = _empty(spatial_index_bytes(nb, n), dtype=torch.uint8, device=xyz.device)
        gidx, geom, kx = knn_group_indexed(sampled, xyz, k, ws, out=kout)
    else:
        gidx, geom, kx = knn_group(sampled, xyz, k, out=kout)
    _record_knn(f"knn_{lvl + 1}", gidx, nb, n, k, True)
    return idx, sampled, gidx, geom, kx


def alloc_stage1(B: int, N: int, device):
    """Buffers of the input-only stage: points [2B,N,3] + level-1 grouping outputs."""
    nb = 2 * B
    M, k = LEVELS[0][:2]
    R = nb * M * k
    ws = _empty(max(spatial_index_bytes(nb, N), 16), dtype=torch.uint8, device=device)
    return (_empty(nb, N, 3, device=device),
            (_empty(nb, M, dtype=torch.int32, device=device), _empty(nb, M, 3, device=device),
             _empty(R, dtype=torch.int32, device=device), _empty(R, 4, device=device),
             _empty(R, 3, device=device), ws))


def stage1_into(bufs, src, dst):
    """cat(src, dst) + level-1 FPS + knn_group into preallocated buffers."""
    pts, g = bufs
    torch.cat([src, dst], 0, out=pts)
    grouping(pts, 0, out=g, ws=g[5])


def _fused23_kernel(P: PreparedWeights, lvl: int):
    """The fused level-2/3 kernel's entry point, weight table and whether it is a bf16x6 one
    (its input projection then uses the bf16x6 table too)."""
    split = (SPLIT_L2, SPLIT_L3)[lvl - 1]
    if lvl == 1 and B6_L2 and not SPLIT_L2:
        name, table = "hreg_group6_l2", P.l2_table6
    elif lvl == 2 and B6_L3 and not SPLIT_L3:
        name, table = "hreg_group6_l3", P.l3_table6
    elif split and (B6_L2, B6_L3)[lvl - 1]:
        name, table = (("hreg_group_split6_l2", P.l2s_table6) if lvl == 1 else
                       ("hreg_group_split6_l3", P.l3s_table6))
    elif split:
        name, table = (("hreg_group_split_l2", P.l2s_table) if lvl == 1 else
                       ("hreg_group_split_l3", P.l3s_table))
    else:
        name, table = (("hreg_group_l2", P.l2_table) if lvl == 1 else
                       ("hreg_group_l3", P.l3_table))
    b6 = name in ("hreg_group6_l2", "hreg_group6_l3", "hreg_group_split6_l2",
                  "hreg_group_split6_l3")
    return name, table, b6


def keypoint_level(P: PreparedWeights, lvl: int, xyz, feats, weights, grouped=None, sample=None):
    """KeypointDetector (layers.py:134-165) + DescExtractor (layers.py:200-209) for one level.

    xyz [nb,n,3]; feats [nb*n, Cf] point-major or None; weights [nb*n] or None;
    grouped: this level's grouping() result when computed ahead (pipelined level 1).
    Returns keypoints [nb,M,3], sigmas [nb*M], att_feat [nb*M,Cdet], desc [nb*M,Cdesc],
    next weights [nb*M] (or None) and the FPS indices [nb,M].
    """
    M, k, Cf, _, _, _ = LEVELS[lvl]
    nb, n, _ = xyz.shape
    G = nb * M
    R = G * k
    fused23 = (lvl == 1 and FUSED_L2) or (lvl == 2 and FUSED_L3)
    pre = None
    fk = _fork_begin() if (grouped is None and fused23 and LEVEL_PRE and _fork_on) else None
    if fk is not None:
        # (chain_fork) the level's input projection beside its WFPS + kNN
        name, table, b6 = _fused23_kernel(P, lvl)
        lin = (P.level_pre6 if b6 else P.level_pre)[lvl]
        pre = _empty(feats.shape[0], lin.N, device=feats.device)
        main, side = fk
        with torch.cuda.stream(side):
            gemm([_seg(feats, 0, Cf)], lin, feats.shape[0], out=pre)
        grouped = grouping(xyz, lvl, weights, sample=sample)
        main.wait_stream(side)
    elif grouped is None:
        grouped = grouping(xyz, lvl, weights, sample=sample)
    idx, sampled, gidx, geom, kx = grouped[:5]
    if lvl == 0 and FUSED_L1:
        dev = xyz.device
        kp = _empty(G, 3, device=dev)
        att_feat = _empty(G, LEVELS[0][3][-1], device=dev)
        desc = _empty(G, LEVELS[0][5], device=dev)
        if B6_L1:
            call("hreg_group_l1_6" if n <= L1_LDS_MAX_N else "hreg_group_l1_6g", P.l1_table6, geom, kx, G, kp,
                 att_feat, desc, _stream())
        else:
            call("hreg_group_l1", P.l1_table, geom, kx, G, kp, att_feat, desc, _stream())
        sig, wnext = mlp_head(P, ("det", lvl), att_feat, nb, M, _lib.HREG_HEAD_SOFTPLUS,
                              want_weights=True)
        return kp.view(nb, M, 3), sig, att_feat, desc, wnext, idx
    if fused23:
        dev = xyz.device
        kp = _empty(G, 3, device=dev)
        att_feat = _empty(G, LEVELS[lvl][3][-1], device=dev)
        desc = _empty(G, LEVELS[lvl][5], device=dev)
        name, table, b6 = _fused23_kernel(P, lvl)
        if pre is None and LEVEL_PRE:
            pre = gemm([_seg(feats, 0, Cf)], (P.level_pre6 if b6 else P.level_pre)[lvl], feats.shape[0])
        if name == "hreg_group_split6_l3" and pre is not None and SPLIT_JT:
            name = "hreg_group_split6j_l3"
        call(name, table, geom, kx, gidx, feats, G, kp, att_feat, desc, pre, _stream())
        sig, wnext = mlp_head(P, ("det", lvl), att_feat, nb, M, _lib.HREG_HEAD_SOFTPLUS,
                              want_weights=True)
        return kp.view(nb, M, 3), sig, att_feat, desc, wnext, idx
    segs = [_seg(geom, 0, 4)]
    if feats is not None:
        segs.append(_seg(feats, 4, Cf, gather=gidx))
    # detector convs (layers.py:150)
    h = gemm(segs, P.det[lvl][0], R)
    h = gemm([_seg(h, 0, h.shape[1])], P.det[lvl][1], R)
    emb = gemm([_seg(h, 0, h.shape[1])], P.det[lvl][2], R)
    attw, att_feat, kp = attend(emb, G, k, vals=emb, xyz_rows=kx, want_attw=True)
    sig, wnext = mlp_head(P, ("det", lvl), att_feat, nb, M, _lib.HREG_HEAD_SOFTPLUS,
                          want_weights=True)
    # descriptor (layers.py:200-209)
    x = gemm(segs, P.desc[lvl][0], R)
    x = gemm([_seg(x, 0, x.shape[1])], P.desc[lvl][1], R)
    x1 = gemm([_seg(x, 0, x.shape[1])], P.desc[lvl][2], R)
    C1 = x1.shape[1]
    x2 = group_max(x1, G, k)
    Cd = emb.shape[1]
    y = gemm([_seg(x2, 0, C1, row_div=k), _seg(x1, C1, C1),
              _seg(emb, 2 * C1, Cd, rowscale=attw)], P.desc_mlp[lvl][0], R)
    y = gemm([_seg(y, 0, y.shape[1])], P.desc_mlp[lvl][1], R)
    desc = group_max(y, G, k)
    return kp.view(nb, M, 3), sig, att_feat, desc, wnext, idx


def feature_extraction(P: PreparedWeights, points, use_weights=True, l1=None, samples=None):
    """HierFeatureExtraction.forward (models.py:26-58) over nb clouds at once.
    l1: level-1 grouping computed ahead (see Pipeline); samples: per-level random-sampling
    indices (use_fps=False, random_samples), else FPS / WFPS."""
    out = {}
    xyz, feats, w = points, None, None
    for lvl in range(3):
        kp, sig, att, desc, wnext, idx = keypoint_level(P, lvl, xyz, feats, w,
                                                        l1 if lvl == 0 else None,
                                                        None if samples is None else samples[lvl])
        out[f"xyz_{lvl + 1}"] = kp
        out[f"sigmas_{lvl + 1}"] = sig
        out[f"desc_{lvl + 1}"] = desc
        out[f"fps_idx_{lvl + 1}"] = idx
        xyz, feats = kp, att
        w = wnext if use_weights else None
    return out


def _head_layers(P: PreparedWeights, key):
    if key == "coarse":
        return P.coarse_head
    if isinstance(key, tuple):
        return P.det_head[key[1]]
    return P.fine[key][1]


def mlp_head(P: PreparedWeights, key, x, nclouds, rows, mode, want_weights=False):
    """mlp1 -> mlp2 -> mlp3 + softplus(+0.001) / sigmoid over per-keypoint rows x
    [nclouds*rows][C] (layers.py:124-132,161-163; 262-268,389-394; 425-431,451-452).
    key: ("det", lvl), "coarse" or the FineReg name.  One mlp_head.hip launch, or
    with FUSED_HEAD off two GEMMs + hreg_head_out.  Returns (out, weights or None)."""
    C = x.shape[1]
    if FUSED_HEAD and C in (64, 128, 256, 512) and (nclouds * rows) % 32 == 0:
        dev = x.device
        out = _empty(nclouds * rows, device=dev)
        wout = _empty(nclouds * rows, device=dev) if want_weights else None
        if B6_MLP:
            # (chain_fork: a forward alone) one row tile per workgroup -- a batch-8 head is 32-128
            # workgroups at the default 2-4 tiles each
            call("hreg_mlp_head6x", P.head_table6[key], C, x, C, nclouds, rows, mode, out, wout,
                 1 if _fork_on else 0, _stream())
        else:
            call("hreg_mlp_head", P.head_table[key], C, x, C, nclouds, rows, mode, out, wout,
                 _stream())
        return out, wout
    m1, m2, w3, b3 = _head_layers(P, key)
    G = nclouds * rows
    s = gemm([_seg(x, 0, C)], m1, G)
    s = gemm([_seg(s, 0, s.shape[1])], m2, G)
    return head_out(s, s.shape[1], nclouds, rows, w3, b3, mode, want_weights=want_weights)


def _mlp_weights(P: PreparedWeights, key, x, nclouds, rows):
    w, _ = mlp_head(P, key, x, nclouds, rows, _lib.HREG_HEAD_SIGMOID)
    return w


# The registration heads' products of the feature-extraction outputs -- CoarseReg's neighbour
# branch block (W_desc desc3), its convs_1 desc / knn_desc blocks, the original cosine
# similarity, and both FineReg heads' descriptor blocks -- depend on nothing but desc_1..3, so
# they run as ONE grouped launch right after the feature extraction (hreg_gemm_grouped: the
# same bits as five separate hreg_gemm launches, one launch instead of five small ones; test
# checker: False, the separate launches)
GROUPED_HEAD_GEMMS = True


def _grouped_heads_ok(C3: int) -> bool:
    return (GROUPED_HEAD_GEMMS and FUSED_NBR and HEAD_PRE and B6_HEADS and COARSE_SPLIT and
            FUSED_COARSE and FUSED_FINE and C3 == 256)


def head_products(P: PreparedWeights, B: int, desc):
    """desc = [desc_1, desc_2, desc_3] (each [2B*M][C], src rows then dst rows) -> the products
    coarse_reg / fine_reg would compute (see GROUPED_HEAD_GEMMS), from one launch."""
    d3 = desc[2]
    dev = d3.device
    C = d3.shape[1]
    N1 = d3.shape[0] // (2 * B)
    norms = row_norms(d3)
    nbr_pre = _empty(2 * B * N1, P.nbr_pre6.N, device=dev)
    ud = _empty(2, B * N1, P.coarse_c1_desc6.W.shape[1], device=dev)
    S = _empty(B, N1, N1, device=dev)
    gs = [_gemm_struct([_seg(d3, 0, C)], P.nbr_pre6, 2 * B * N1, nbr_pre),
          _batched_desc_struct(P.coarse_c1_desc6, d3, B * N1, C, ud),
          _cosine_struct(d3[:B * N1], d3[B * N1:], norms[:B * N1], norms[B * N1:], B, N1, N1, C, S)]
    fine = {}
    for name, lv in (("fine_corres_2", 1), ("fine_corres_1", 0)):
        dl = desc[lv]
        M, Cl = dl.shape[0] // (2 * B), dl.shape[1]
        pre = _empty(2, B * M, P.fine[name][0][0].W.shape[0], device=dev)
        gs.append(_batched_desc_struct(P.fine_pre6[name], dl, B * M, Cl, pre))
        fine[name] = pre
    _lib.gemm_grouped(gs)
    return {"nbr_pre": nbr_pre, "ud": ud, "S": S, "fine_pre": fine}


def coarse_knns(B, xyz3, desc3, out=None):
    """CoarseReg's two kNN selections, which depend on the level-3 keypoints only: the
    descriptor-space kNN src -> dst (layers.py:278) and the xyz kNN of every keypoint among its
    own cloud's (layers.py:315-337).  out: (kidx, (gidx, geom, kx)) preallocated."""
    k = K_HEAD
    N1 = xyz3.shape[1]
    C = desc3.shape[1]
    s_desc, d_desc = desc3[:B * N1], desc3[B * N1:]
    kidx = knn_idx32(s_desc.view(B, N1, C), d_desc.view(B, N1, C), k, out=None if out is None else out[0])
    g = knn_group(xyz3, xyz3, k, out=None if out is None else out[1])
    return kidx, g


def coarse_knns_alloc(B, xyz3):
    dev = xyz3.device
    N1 = xyz3.shape[1]
    R2 = 2 * B * N1 * K_HEAD
    return (_empty(B, N1, K_HEAD, dtype=torch.int32, device=dev),
            (_empty(R2, dtype=torch.int32, device=dev), _empty(R2, 4, device=dev), _empty(R2, 3, device=dev)))


def coarse_reg(P: PreparedWeights, B, xyz3, desc3, sig3, prod=None, knns=None):
    """CoarseReg.forward (layers.py:273-396); xyz3 [2B,256,3], desc3 [2B*256,256], sig3 [2B*256].
    prod: head_products' precomputed blocks and original similarity (else computed here);
    knns: coarse_knns' result computed ahead (else computed here).  Under chain_fork() the
    neighbour head runs on a side stream beside the first similarity gather."""
    dev = xyz3.device
    k = K_HEAD
    N1 = xyz3.shape[1]
    C = desc3.shape[1]
    s_desc, d_desc = desc3[:B * N1], desc3[B * N1:]
    s_xyz, d_xyz = xyz3[:B], xyz3[B:]
    s_sig, d_sig = sig3[:B * N1], sig3[B * N1:]
    # desc-space kNN (layers.py:278) and the keypoints' own-cloud kNN (layers.py:315-337)
    kidx, (gself, geom_self, _) = knns if knns is not None else coarse_knns(B, xyz3, desc3)
    _record_knn("coarse_desc_knn", kidx, B, N1, k, False)
    _record_knn("coarse_nbr", gself, 2 * B, N1, k, True)
    G2 = 2 * B * N1
    R2 = G2 * k
    b6 = B6_HEADS and HEAD_PRE
    # (chain_fork) the fused neighbour head beside the first similarity gather
    use_sim, use_nbr = P.coarse_use_sim, P.coarse_use_nbr
    fk = (_fork_begin() if (_fork_on and use_nbr and prod is not None and FUSED_NBR and C == 256 and b6
                            and SPLIT_NBR) else None)
    if fk is not None:
        nbr = _empty(G2, C, device=dev)
        main, side = fk
        with torch.cuda.stream(side):
            call("hreg_nbr_head6sx", P.nbr_table6, desc3, gself, geom_self, G2, nbr, prod["nbr_pre"],
                 HEAD_ROW_TILES, _stream())
    # original similarity (layers.py:290-313)
    if prod is not None:
        S = prod["S"]
    else:
        norms = row_norms(desc3)
        S = _empty(B, N1, N1, device=dev)
        cosine_gemm(s_desc, d_desc, norms[:B * N1], norms[B * N1:], B, N1, N1, C, S)
    maxes = _empty(B, 2 * N1, device=dev)
    if use_sim:
        sims_a = _empty(B * N1 * k, 2, device=dev)
        call("hreg_sim_gather", S, B, N1, N1, kidx, k, maxes, sims_a, 2, _stream())
    else:  # (variant: zero features under zero weight columns, _pad_coarse_convs1)
        sims_a = torch.zeros(B * N1 * k, 2, device=dev)
    # neighbour-aware descriptors for src and dst together (layers.py:315-337)
    if not use_nbr:
        nbr = None
    elif fk is not None:
        main.wait_stream(side)
    elif FUSED_NBR and C == 256:
        nbr = _empty(G2, C, device=dev)
        if prod is not None:
            pre = prod["nbr_pre"]
        else:
            pre = gemm([_seg(desc3, 0, C)], P.nbr_pre6 if b6 else P.nbr_pre, G2) if HEAD_PRE else None
        if b6:
            if SPLIT_NBR:
                call("hreg_nbr_head6sx", P.nbr_table6, desc3, gself, geom_self, G2, nbr, pre, HEAD_ROW_TILES,
                     _stream())
            else:
                call("hreg_nbr_head6", P.nbr_table6, desc3, gself, geom_self, G2, nbr, pre, _stream())
        else:
            call("hreg_nbr_head", P.nbr_table, desc3, gself, geom_self, G2, nbr, pre, _stream())
    else:
        segs = [_seg(desc3, 0, C, gather=gself), _seg(geom_self, C, 4)]
        h = gemm(segs, P.coarse_convs2[0], R2)
        h = gemm([_seg(h, 0, h.shape[1])], P.coarse_convs2[1], R2)
        h = gemm([_seg(h, 0, h.shape[1])], P.coarse_convs2[2], R2)
        _, nbr, _ = attend(h, G2, k, vals=desc3, vgather=gself)
    if use_nbr:
        nnorm = row_norms(nbr)
        cosine_gemm(nbr[:B * N1], nbr[B * N1:], nnorm[:B * N1], nnorm[B * N1:], B, N1, N1, C, S)
        sims_b = _empty(B * N1 * k, 2, device=dev)
        call("hreg_sim_gather", S, B, N1, N1, kidx, k, maxes, sims_b, 2, _stream())
    else:
        sims_b = torch.zeros(B * N1 * k, 2, device=dev)
    # correspondence features + convs_1 (layers.py:364-384)
    R = B * N1 * k
    small = _empty(R, 16, device=dev)
    kx = _empty(R, 3, device=dev)
    gidx = _empty(R, dtype=torch.int32, device=dev)
    call("hreg_pair_feats", s_xyz, d_xyz, s_sig, d_sig, kidx, B, N1, N1, k, sims_a, sims_b,
         small, 16, kx, gidx, _stream())
    if COARSE_SPLIT:
        # W [small | desc | knn_desc]: the desc block is the same for the k rows of a
        # keypoint and the knn_desc block the same for every row gathering that dst
        # keypoint, so both are multiplied once per keypoint (one batch-2 GEMM over
        # desc3 = [src; dst]) and added in the layer's epilogue: 8.86 -> 1.34 GFLOP
        # per step at B=8 for this layer
        fused = FUSED_COARSE and C == 256
        if prod is not None:
            ud = prod["ud"]
        else:
            ud = _empty(2, B * N1, P.coarse_c1_desc.W.shape[1], device=dev)
            _gemm_batched_desc(P.coarse_c1_desc6 if fused else P.coarse_c1_desc, desc3, B * N1, C, ud)
        if fused:
            # convs_1 + attention in one launch (coarse6.hip)
            corres = _empty(B * N1, 3, device=dev)
            att = _empty(B * N1, ud.shape[2], device=dev)
            call("hreg_coarse_head6", P.coarse_table6, small, ud[0], ud[1], gidx, kx, B * N1,
                 corres, att, _stream())
            w = _mlp_weights(P, "coarse", att, B, N1)
            return corres.view(B, N1, 3), w.view(B, N1)
        f = gemm([_seg(small, 0, 16)], P.coarse_c1_small, R,
                 adds=[_seg(ud[0], 0, 4, row_div=k), _seg(ud[1], 0, 4, gather=gidx)])
    else:
        segs = [_seg(small, 0, 16), _seg(s_desc, 16, C, row_div=k),
                _seg(d_desc, 16 + C, C, gather=gidx)]
        f = gemm(segs, P.coarse_convs1[0], R)
    f = gemm([_seg(f, 0, f.shape[1])], P.coarse_convs1[1], R, b6=True)
    f = gemm([_seg(f, 0, f.shape[1])], P.coarse_convs1[2], R, b6=True)
    _, att, corres = attend(f, B * N1, k, vals=f, xyz_rows=kx)
    w = _mlp_weights(P, "coarse", att, B, N1)
    return corres.view(B, N1, 3), w.view(B, N1)


def fine_reg(P: PreparedWeights, name, B, src_xyz, src_desc, dst_xyz, dst_desc, src_w, dst_w,
             return_att=False, pre=None):
    """FineReg.forward (layers.py:433-454); xyz [B,N,3], desc [B*N,C], w [B*N].
    pre: the descriptor blocks head_products made (else computed here)."""
    dev = src_xyz.device
    k = K_HEAD
    N = src_xyz.shape[1]
    C = src_desc.shape[1]
    convs, head = P.fine[name]
    kidx = knn_idx32(src_xyz, dst_xyz, k)
    _record_knn(name + "_knn", kidx, B, dst_xyz.shape[1], k, False)
    R = B * N * k
    if FUSED_FINE:
        small = _empty(R, 16, device=dev)
        kx = _empty(R, 3, device=dev)
        gidx = _empty(R, dtype=torch.int32, device=dev)
        call("hreg_pair_feats", src_xyz, dst_xyz, src_w, dst_w, kidx, B, N, N, k, None, None, small,
             16, kx, gidx, _stream())
        N1 = convs[0].W.shape[0]
        corres = _empty(B * N, 3, device=dev)
        att = _empty(B * N, N1, device=dev)
        if pre is None:
            pre = [None, None]
            if HEAD_PRE:
                pre = _empty(2, B * N, N1, device=dev)
                _gemm_batched_desc((P.fine_pre6 if B6_HEADS else P.fine_pre)[name], src_desc, B * N, C,
                                   pre, x1=dst_desc)
        if B6_HEADS and HEAD_PRE and SPLIT_FINE:
            call("hreg_corr_head6x", P.fine_table6[name], N1, small, pre[0], pre[1], gidx, kx, B * N,
                 corres, att, HEAD_ROW_TILES, _stream())
        elif B6_HEADS and HEAD_PRE:
            call("hreg_fine_head6", P.fine_table6[name], C, small, gidx, kx, B * N, corres, att,
                 pre[0], pre[1], _stream())
        else:
            call("hreg_fine_head", P.fine_table[name], C, small, src_desc, dst_desc, gidx, kx,
                 B * N, corres, att, pre[0], pre[1], _stream())
        w = _mlp_weights(P, name, att, B, N)
        if return_att:
            return corres.view(B, N, 3), w.view(B, N), att
        return corres.view(B, N, 3), w.view(B, N)
    small = _empty(R, 12, device=dev)
    kx = _empty(R, 3, device=dev)
    gidx = _empty(R, dtype=torch.int32, device=dev)
    call("hreg_pair_feats", src_xyz, dst_xyz, src_w, dst_w, kidx, B, N, N, k, None, None, small, 12,
         kx, gidx, _stream())
    segs = [_seg(small, 0, 12), _seg(src_desc, 12, C, row_div=k), _seg(dst_desc, 12 + C, C, gather=gidx)]
    f = gemm(segs, convs[0], R)
    f = gemm([_seg(f, 0, f.shape[1])], convs[1], R)
    f = gemm([_seg(f, 0, f.shape[1])], convs[2], R)
    _, att, corres = attend(f, B * N, k, vals=f, xyz_rows=kx)
    w = _mlp_weights(P, name, att, B, N)
    if return_att:
        return corres.view(B, N, 3), w.view(B, N), att
    return corres.view(B, N, 3), w.view(B, N)


def weighted_svd(src, corres, w, prev=None, group=None, move=None):
    """WeightedSVDHead (layers.py:469-504) (+ T = T_ @ T_prev, models.py:100-127).  group:
    the pairs are batches of `group` pairs merged into one call (the identity fallback of
    layers.py:485-493 per batch); None = one batch.  move [B, n2, 3]: points to move by the
    final R, t in the same launches (hreg_weighted_svd_tr; the next FineReg stage's src
    keypoints) -> (R_, t_, R, t, moved) instead of (R_, t_, R, t)."""
    B, n, _ = src.shape
    dev = src.device
    R_ = _empty(B, 3, 3, device=dev)
    t_ = _empty(B, 3, device=dev)
    R = _empty(B, 3, 3, device=dev)
    t = _empty(B, 3, device=dev)
    pR, pt = (prev if prev is not None else (None, None))
    if move is not None:
        if group is not None and B % group:
            raise ValueError(f"weighted_svd: {B} pairs are not whole batches of {group}")
        moved = torch.empty_like(move)
        call("hreg_weighted_svd_tr", src, corres, w, B, B if group is None else group, n, pR, pt, R_, t_, R, t,
             move, move.shape[1], moved, _stream())
        return R_, t_, R, t, moved
    if group is None or group == B:
        call("hreg_weighted_svd", src, corres, w, B, n, pR, pt, R_, t_, R, t, _stream())
    else:
        if B % group:
            raise ValueError(f"weighted_svd: {B} pairs are not whole batches of {group}")
        call("hreg_weighted_svd_grouped", src, corres, w, B, group, n, pR, pt, R_, t_, R, t, _stream())
    return R_, t_, R, t


def transform(xyz, R, t):
    B, n, _ = xyz.shape
    out = torch.empty_like(xyz)
    call("hreg_transform_points", xyz, R, t, B, n, out, _stream())
    return out


def level_input_sizes(N: int):
    """points entering each level's sampling: the cloud, then the previous level's keypoints"""
    return (N, LEVELS[0][0], LEVELS[1][0])


def hregnet_forward(P: PreparedWeights, src, dst, use_weights=True, l1=None, pts=None, v2=False,
                    use_fps=True, sub_batch=None):
    """HRegNet.forward (models/HRegNet/models.py:77-148), eval mode.

    v2: the Model_V2 variant (models/model_v2/models.py:77-183): fine_corres_2 is
    FineReg2 (model_v2/layers.py:462-500), whose attentive features also pass
    through mlpx (Conv1d 2C->C + BN + ReLU) -> "src_dst_feats_2" [B, C, M2]; the
    batch-shuffled prime copies are added by model_v2_finish (host RNG).

    sub_batch: src / dst are B / sub_batch reference batches of sub_batch pairs merged into one
    launch set (an executor choice: every pair's result is bitwise the same as in its own
    batch's forward -- the kernels are batch-independent -- and the one batch-level step, the
    weighted SVD's identity fallback, applies per batch)."""
    return hregnet_back(P, hregnet_front(P, src, dst, use_weights, l1, pts, use_fps), src.shape[0], v2,
                        sub_batch)


def hregnet_front(P: PreparedWeights, src, dst, use_weights=True, l1=None, pts=None, use_fps=True):
    """The feature extraction of both clouds of HRegNet.forward (models.py:79-80): the
    dict hregnet_back continues from (GraphPipeline runs the two halves of a forward in
    consecutive rounds)."""
    B, N, _ = src.shape
    if pts is None:
        pts = torch.cat([src, dst], 0).contiguous()
    samples = None
    if not use_fps:
        if l1 is not None:
            raise ValueError("use_fps=False draws its level-1 sample in the forward (no l1)")
        samples = random_samples(2, B, level_input_sizes(N), src.device)
    return feature_extraction(P, pts, use_weights, l1, samples)


# what hregnet_back reads of the feature-extraction dict
FRONT_KEYS = tuple(f"{k}_{i + 1}" for k in ("xyz", "sigmas", "desc", "fps_idx") for i in range(3))


def hregnet_back(P: PreparedWeights, fe, B: int, v2=False, sub_batch=None):
    """The registration half of HRegNet.forward (models.py:82-148) from hregnet_front's dict."""

    def split(t, rows):
        return t[:B * rows], t[B * rows:]

    M = [lv[0] for lv in LEVELS]
    xyz = [fe[f"xyz_{i + 1}"] for i in range(3)]
    sig = [fe[f"sigmas_{i + 1}"] for i in range(3)]
    desc = [fe[f"desc_{i + 1}"] for i in range(3)]
    grouped = _grouped_heads_ok(desc[2].shape[1])
    # (chain_fork) CoarseReg's kNN selections beside the grouped head products
    fk = _fork_begin() if (_fork_on and grouped) else None
    knns = None
    if fk is not None:
        knns = coarse_knns_alloc(B, xyz[2])
        main, side = fk
        with torch.cuda.stream(side):
            coarse_knns(B, xyz[2], desc[2], out=knns)
    prod = head_products(P, B, desc) if grouped else None
    if fk is not None:
        main.wait_stream(side)
    fpre = (lambda name: None) if prod is None else (lambda name: prod["fine_pre"][name])
    c3, w3 = coarse_reg(P, B, xyz[2], desc[2], sig[2], prod, knns=knns)
    # (the src level-2 keypoints moved by (R3, t3) in the SVD's batch launch)
    _, _, R3, t3, x2t = weighted_svd(xyz[2][:B], c3, w3, group=sub_batch, move=xyz[1][:B])
    sd2, dd2 = split(desc[1], M[1])
    ss2, ds2 = split(sig[1], M[1])
    if v2:
        if P.mlpx is None:
            raise RuntimeError("Model_V2 forward: the state dict has no fine_corres_2.mlpx")
        c2, w2, att2 = fine_reg(P, "fine_corres_2", B, x2t, sd2, xyz[1][B:], dd2, ss2, ds2,
                                return_att=True, pre=fpre("fine_corres_2"))
        f2 = gemm([_seg(att2, 0, att2.shape[1])], P.mlpx, B * M[1])
    else:
        c2, w2 = fine_reg(P, "fine_corres_2", B, x2t, sd2, xyz[1][B:], dd2, ss2, ds2,
                          pre=fpre("fine_corres_2"))
    _, _, R2, t2, x1t = weighted_svd(x2t, c2, w2, prev=(R3, t3), group=sub_batch, move=xyz[0][:B])
    sd1, dd1 = split(desc[0], M[0])
    ss1, ds1 = split(sig[0], M[0])
    c1, w1 = fine_reg(P, "fine_corres_1", B, x1t, sd1, xyz[0][B:], dd1, ss1, ds1,
                      pre=fpre("fine_corres_1"))
    _, _, R1, t1 = weighted_svd(x1t, c1, w1, prev=(R2, t2), group=sub_batch)

    def feats(part):
        sl = slice(0, B) if part == 0 else slice(B, 2 * B)
        d = {}
        for i in range(3):
            m = M[i]
            d[f"xyz_{i + 1}"] = xyz[i][sl]
            d[f"sigmas_{i + 1}"] = sig[i].view(2 * B, m)[sl]
            d[f"desc_{i + 1}"] = desc[i].view(2 * B, m, -1)[sl].transpose(1, 2)
        return d

    out = {
        "src_xyz_corres_3": c3, "src_xyz_corres_2": c2, "src_xyz_corres_1": c1,
        "src_dst_weights_3": w3, "src_dst_weights_2": w2, "src_dst_weights_1": w1,
        "rotation": [R3, R2, R1], "translation": [t3, t2, t1],
        "src_feats": feats(0), "dst_feats": feats(1),
        "_fps_idx": [fe[f"fps_idx_{i + 1}"] for i in range(3)],
    }
    if v2:
        out["src_xyz_2_trans"] = x2t
        out["src_dst_feats_2"] = f2.view(B, M[1], -1).transpose(1, 2)
    return out


def model_v2_finish(out, sub_batch=None):
    """The Model_V2 result dict (models/model_v2/models.py:145-183) from
    hregnet_forward(..., v2=True): the "prime" copies are batch shuffles drawn with
    torch.randperm(B) on the default (host) generator, features first, then weights
    (model_v2/layers.py:491-497), as the reference draws them.  sub_batch (merged batches,
    hregnet_forward): each batch of sub_batch pairs is shuffled within itself, its two draws
    in batch order -- the draws of the forwards of those batches one after another."""
    f2, w2 = out["src_dst_feats_2"], out["src_dst_weights_2"]
    B = w2.shape[0]
    sb = B if sub_batch is None else sub_batch
    if B % sb:
        raise ValueError(f"model_v2_finish: {B} pairs are not whole batches of {sb}")
    pfs, pws = [], []
    for b0 in range(0, B, sb):
        pfs.append(torch.randperm(sb) + b0)
        pws.append(torch.randperm(sb) + b0)
    pf = torch.cat(pfs)
    pw = torch.cat(pws)
    sf, df = out["src_feats"], out["dst_feats"]
    return {
        "src_xyz_corres_3": out["src_xyz_corres_3"], "src_xyz_corres_2": out["src_xyz_corres_2"],
        "src_xyz_corres_1": out["src_xyz_corres_1"],
        "rotation": out["rotation"], "translation": out["translation"],
        "src_feats_desc_2": sf["desc_2"], "src_feats_sigmas_2": sf["sigmas_2"],
        "src_xyz_2_trans": out["src_xyz_2_trans"], "dst_xyz_2": df["xyz_2"],
        "src_dst_feats_2": f2, "src_dst_feats_2_prime": f2[pf.to(f2.device)],
        "src_dst_weights_2": w2, "src_dst_weights_2_prime": w2[pw.to(w2.device)],
        "src_feats": sf, "dst_feats": df,
        "_fps_idx": out["_fps_idx"],
    }


def model_v2_forward(P: PreparedWeights, src, dst, use_weights=True, use_fps=True):
    """Model_V2.forward (models/model_v2/models.py:77-183), eval mode."""
    return model_v2_finish(hregnet_forward(P, src, dst, use_weights, v2=True, use_fps=use_fps))


class Pipeline:
    """Throughput executor: level-1 FPS + kNN grouping of batch i+1 runs on a side
    stream while the rest of batch i runs on the caller's stream.

    Level 1 depends only on the input points, and FPS is a serial 1023-step
    chain on one CU per cloud (2B CUs busy), so overlapping it with the
    previous batch's GEMM-heavy levels hides it.  Every batch still goes
    through the complete forward; results are identical to hregnet_forward.
    """

    def __init__(self, P: PreparedWeights, device, v2: bool = False, sub_batch=None):
        self.P = P
        self.v2 = v2
        self.sub_batch = sub_batch  # (hregnet_forward's merged reference batches)
        self.side = torch.cuda.Stream(device=device)

    def _stage1(self, src, dst):
        pts = torch.cat([src, dst], 0).contiguous()
        return pts, grouping(pts, 0)

    def run(self, batches, use_weights=True):
        """batches: iterable of (src [B,N,3], dst [B,N,3]) on the GPU -> list of output dicts."""
        main = torch.cuda.current_stream()
        ev_in = torch.cuda.Event()
        ev_in.record(main)
        self.side.wait_event(ev_in)
        batches = list(batches)
        pending = []

        def launch(i):
            src, dst = batches[i]
            with torch.cuda.stream(self.side):
                pts, g = self._stage1(src, dst)
                ev = torch.cuda.Event()
                ev.record(self.side)
            for t in (src, dst):
                t.record_stream(self.side)
            pending.append((pts, g, ev))

        outs = []
        if batches:
            launch(0)
        for i, (src, dst) in enumerate(batches):
            if i + 1 < len(batches):
                launch(i + 1)
            pts, g, ev = pending.pop(0)
            main.wait_event(ev)
            pts.record_stream(main)
            for t in g:
                t.record_stream(main)
            out = hregnet_forward(self.P, src, dst, use_weights, l1=g, pts=pts, v2=self.v2,
                                  sub_batch=self.sub_batch)
            outs.append(model_v2_finish(out, self.sub_batch) if self.v2 else out)
        check_device_status()  # syncs only when a multi-workgroup FPS ran
        return outs


# GPU_MAX_HW_QUEUES (HIP's hardware queues per process, default 4) the graph executor has run
# on: 4, 8 and 16 (DESIGN.md section 10, r4 queue sweep).  With 2 the r4 bench process died in
# the HIP runtime (core dump, gpurun_out/hwq/q2.s20.1.err) while replaying a round of 20 lanes
# whose graph forks 2 x 20 + 1 streams (lane stream, front stream, the batched stage-1 stream).
# Nothing in the graph needs more than one queue for correctness (every cross-stream order is a
# graph edge), so the crash is the runtime's, not a dependency the graph leaves to queue
# order; what the executor can do is not walk into it: fewer queues than MIN_HW_QUEUES are
# refused up front with this error instead of a segfault mid-replay.
MIN_HW_QUEUES = 4


def hw_queues(env=None) -> int:
    """GPU_MAX_HW_QUEUES as the HIP runtime reads it (unset or invalid: its default 4)."""
    import os
    v = (os.environ if env is None else env).get("GPU_MAX_HW_QUEUES", "")
    try:
        q = int(v)
    except ValueError:
        return 4
    return q if q > 0 else 4


def check_hw_queues(streams: int, env=None) -> int:
    """Refuse a graph executor whose fork width (``streams`` concurrent streams per replay)
    would run on fewer hardware queues than have been measured to work; -> the queue count."""
    q = hw_queues(env)
    if q < MIN_HW_QUEUES and streams > 1:
        raise RuntimeError(
            f"GraphPipeline: GPU_MAX_HW_QUEUES={q} with {streams} forked streams per replay; the "
            f"graph executor runs on >= {MIN_HW_QUEUES} hardware queues (measured 4, 8, 16; 2 "
            "crashed the HIP runtime in r4). Unset GPU_MAX_HW_QUEUES or set it to 4.")
    return q


def fork_width(lanes: int, batched_stage1: bool, front_two_streams: bool) -> int:
    """Streams one replay of the executor forks: a stream per lane (lane 0 the capture
    stream), a second per lane for the front half, and the stage-1 side
    stream(s) -- one batched, or one per lane."""
    return lanes * (2 if front_two_streams else 1) + (1 if batched_stage1 else lanes)


def copy_many(dsts, srcs) -> None:
    """dst.copy_(src) for each pair (same dtype and shape, contiguous) in one hreg_copy_many launch
    per 16 pairs; any other pair through torch"""
    import ctypes
    pairs = [(d, s) for d, s in zip(dsts, srcs)
             if d.is_contiguous() and s.is_contiguous() and d.dtype == s.dtype and d.shape == s.shape
             and (d.numel() * d.element_size()) % 4 == 0]
    rest = [(d, s) for d, s in zip(dsts, srcs) if not any(d is p for p, _ in pairs)]
    for i in range(0, len(pairs), 16):
        chunk = pairs[i:i + 16]
        n = len(chunk)
        src = (ctypes.c_void_p * n)(*[s.data_ptr() for _, s in chunk])
        dst = (ctypes.c_void_p * n)(*[d.data_ptr() for d, _ in chunk])
        nb = (ctypes.c_size_t * n)(*[d.numel() * d.element_size() for d, _ in chunk])
        call("hreg_copy_many", n, src, dst, nb, _stream())
    for d, s in rest:
        d.copy_(s)


class GraphPipeline:
    """The pipelined forward captured as HIP graphs (kernel boundaries ~1.5 us
    instead of a host launch each).

    ``lanes`` independent batches are in flight at once, each on its own stream
    inside one graph: the forward is a chain of kernels of very different widths
    (the WFPS levels and the small head GEMMs occupy a handful of CUs for
    hundreds of us, the level-2/3 conv GEMMs fill the chip), so a second batch
    fills one batch's narrow phases.  Per lane: static inputs ``src``/``dst``
    (copy new data in with ``load``) and two level-1 buffer sets A/B.  g_AB =
    {lane side stream: stage 1 of the lane's next batch into B ; lane stream: the
    rest of the forward from A}, g_BA symmetric; replaying them alternately
    overlaps batch i+1's level-1 FPS with batch i.  Every batch runs the
    complete forward; outputs are bitwise those of ``hregnet_forward``.
    v2: the Model_V2 forward; the prime shuffles (host torch.randperm, as the
    reference draws them) are gathered eagerly after each round's replay.

    FRONT_STREAM (batched stage 1, streaming calls of whole rounds): a forward's two halves
    run in consecutive rounds -- round r replays, per lane, the registration half of the
    batch whose feature extraction round r - 1 ran (``hregnet_back``) and, on a second
    stream of the lane, the feature extraction of the next batch (``hregnet_front``, its dict
    copied into static buffers), beside the batched stage 1 of the batch after that.  Every
    round still completes ``lanes`` whole forwards, but each lane's dependent chain per round
    is half a forward, so the round's tail (the last chains draining, ~1.3 ms of a 20-lane
    round) is shorter: +3.2 % at 20 lanes; at 48 lanes, where the tail is 2.5 % of the
    round, it measured ~1 % slower, hence FRONT_STREAM_MAX_LANES.  ``prime()`` fills the pipeline (untimed: the
    bench calls it after its warm-up).
    """

    def __init__(self, P: PreparedWeights, src, dst, use_weights=True, lanes: int = 1,
                 v2: bool = False, sub_batch=None):
        self.P = P
        self.v2 = v2
        # sub_batch: every lane's batch is B / sub_batch reference batches merged into one
        # launch set (hregnet_forward's sub_batch; the bench's Model_V2 line)
        self.sub_batch = sub_batch
        self.use_weights = use_weights
        self.lanes = lanes
        dev = src.device
        B, N, _ = src.shape
        self.B, self.N = B, N
        # BATCH_STAGE1: stage 1 (level-1 FPS + spatial index + kNN) of every lane's next batch
        # as ONE launch each over lanes x 2B clouds on one side stream; the lanes read
        # cloud-slice views of it (the level-1 kernel reads geom / knn_xyz, not the global
        # gidx: FUSED_L1 only)
        # (clouds above 16384 points -- Model_V2's config -- keep the per-lane stage: their
        # multi-workgroup FPS spins every participant of a launch, and one batched launch
        # measured slower: 803 vs 844 pairs/s)
        # (Model_V2's 65536-point clouds, V2_BATCH_STAGE1: one cluster-FPS launch over every
        # lane's clouds with the bounded-concurrency spin budget -- its stream is the only one
        # that runs multi-workgroup FPS -- instead of one launch per lane on per-lane side streams,
        # which shared the 4 hardware queues with the lanes' own streams)
        self.bs1 = BATCH_STAGE1 and FUSED_L1 and lanes > 1 and (N <= 16384 or (v2 and V2_BATCH_STAGE1))
        check_hw_queues(fork_width(lanes, self.bs1, FRONT_STREAM and self.bs1 and not v2
                                   and lanes <= FRONT_STREAM_MAX_LANES))
        if self.bs1:
            self.src_all = src.unsqueeze(0).repeat(lanes, 1, 1, 1).contiguous()
            self.dst_all = dst.unsqueeze(0).repeat(lanes, 1, 1, 1).contiguous()
            self.src = [self.src_all[ln] for ln in range(lanes)]
            self.dst = [self.dst_all[ln] for ln in range(lanes)]
            self.bufs_all = [alloc_stage1(B * lanes, N, dev) for _ in (0, 1)]
            self.bufs = [[self._lane_view(ab, ln) for ab in (0, 1)] for ln in range(lanes)]
        else:
            self.src = [src.clone() for _ in range(lanes)]
            self.dst = [dst.clone() for _ in range(lanes)]
            self.bufs = [[alloc_stage1(B, N, dev), alloc_stage1(B, N, dev)] for _ in range(lanes)]
        self.side = [torch.cuda.Stream(device=dev) for _ in range(lanes)]
        self.lane_streams = [torch.cuda.Stream(device=dev) for _ in range(lanes)]
        # one lane: a forward alone is one dependent chain -- fork what does not depend on it
        # (chain_fork) onto the lane's otherwise unused stream
        with (chain_fork(side=self.lane_streams[0]) if lanes == 1 else contextlib.nullcontext()):
            # eager warm-up: library, allocator and workspace shapes
            if self.bs1:
                self._stage1_all(0)
            else:
                stage1_into(self.bufs[0][0], self.src[0], self.dst[0])
            self._rest(0, 0)
            torch.cuda.synchronize()
            # the captured graphs contain multi-workgroup FPS launches (n > 16384): their
            # device status is checked by check() after replays
            self.status_check = _status_pending
            check_device_status()
            self.pool = torch.cuda.graph_pool_handle()
            self.g_first = torch.cuda.CUDAGraph()
            with capture.graph(self.g_first, pool=self.pool):
                self._first_stage1()
            self.g_step, self.outs = [], []
            for cur in (0, 1):
                g = torch.cuda.CUDAGraph()
                with capture.graph(g, pool=self.pool):
                    out = self._fork(lambda ln: self._rest(ln, cur), **self._side_kw(1 - cur))
                self.g_step.append(g)
                self.outs.append(out)
            self.g_last, self.outs_last = [], []
            for cur in (0, 1):
                g = torch.cuda.CUDAGraph()
                with capture.graph(g, pool=self.pool):
                    out = self._fork(lambda ln: self._rest(ln, cur))
                self.g_last.append(g)
                self.outs_last.append(out)
            self._part = {}
            self.ready = None  # buffer set holding a streamed next-round stage 1 (run_forwards)
            # front streaming: fe[c][ln] = static copies of a lane's feature-extraction dict;
            # fready = c: the fronts for the next round are in fe[1 - c] and its next stage 1
            # in bufs[c], so the next replay is g_fs[c]
            self.fs = (FRONT_STREAM and self.bs1 and not v2
                       and lanes <= FRONT_STREAM_MAX_LANES)
            self.fready = None
            if self.fs:
                with torch.no_grad():
                    pts, g = self.bufs[0][0]
                    fe0 = hregnet_front(P, self.src[0], self.dst[0], use_weights, l1=g, pts=pts)
                self.fe = [[{k: torch.empty_like(fe0[k]) for k in FRONT_KEYS} for _ in range(lanes)]
                           for _ in (0, 1)]
                del fe0
                self.g_fs, self.outs_fs, self.g_prime = [], [], []
                # the two halves of a lane on two streams (r4: 7084 -> 7311 pairs/s, against 7141
                # with both halves on the lane's stream)
                self.lane_streams2 = [torch.cuda.Stream(device=dev) for _ in range(lanes)]
                for cur in (0, 1):
                    g = torch.cuda.CUDAGraph()
                    with capture.graph(g, pool=self.pool):
                        out = self._fork(lambda ln: hregnet_back(P, self.fe[1 - cur][ln], B, v2, sub_batch),
                                         body2=lambda ln: self._front_into(ln, cur), **self._side_kw(1 - cur))
                    self.g_fs.append(g)
                    self.outs_fs.append(out)
                    g = torch.cuda.CUDAGraph()
                    with capture.graph(g, pool=self.pool):
                        self._fork(lambda ln: self._front_into(ln, cur), **self._side_kw(1 - cur))
                    self.g_prime.append(g)
            torch.cuda.synchronize()

    def _lane_view(self, ab: int, ln: int):
        """Lane ln's stage-1 buffers as cloud-slice views of the batched set ab."""
        pts, (idx, sampled, gidx, geom, kx, ws) = self.bufs_all[ab]
        nb = 2 * self.B
        M, k = LEVELS[0][:2]
        R = nb * M * k
        c, r = slice(ln * nb, (ln + 1) * nb), slice(ln * R, (ln + 1) * R)
        return pts[c], (idx[c], sampled[c], gidx[r], geom[r], kx[r], ws)

    def _stage1_all(self, ab: int):
        """Stage 1 of every lane's static batch into buffer set ab: 2 copies + one FPS, one
        spatial index and one kNN launch over lanes x 2B clouds."""
        pts, g = self.bufs_all[ab]
        v = pts.view(self.lanes, 2, self.B, self.N, 3)
        v[:, 0].copy_(self.src_all)
        v[:, 1].copy_(self.dst_all)
        grouping(pts, 0, out=g, ws=g[5], fps_concurrent=1 if self.N > 16384 else 0, fps_lean=FPS_LEAN)

    def _first_stage1(self, lanes=None):
        if self.bs1:
            self._stage1_all(0)
        else:
            self._fork(lambda ln: stage1_into(self.bufs[ln][0], self.src[ln], self.dst[ln]), lanes=lanes)

    def _side_kw(self, ab: int, side_lanes=None):
        """_fork keywords for the next batch's stage 1 into buffer set ab (batched: one job
        for all lanes; per lane: lanes < side_lanes)."""
        if self.bs1:
            return {"side_all": lambda: self._stage1_all(ab)}
        return {"side": lambda ln: stage1_into(self.bufs[ln][ab], self.src[ln], self.dst[ln]),
                "side_lanes": side_lanes}

    def _fork(self, body, side=None, lanes=None, side_lanes=None, side_all=None, body2=None):
        """Inside a capture: body(lane) for every lane < lanes on its own stream (lane 0
        on the capturing stream) and side(lane) for lane < side_lanes on the lane's side
        stream, all forked from the capturing stream and joined back to it (one level of
        fork/join: consecutive graph launches on one stream are ordered, so the side work
        of this launch cannot overlap the previous launch's reads of its buffers).
        Returns the per-lane results of body."""
        main = torch.cuda.current_stream()
        lanes = self.lanes if lanes is None else lanes
        side_lanes = lanes if side_lanes is None else side_lanes
        jobs = []
        if side_all is not None:
            jobs.append((self.side[0], lambda _ln: side_all(), -1))
        for ln in range(lanes):
            if side is not None and ln < side_lanes:
                jobs.append((self.side[ln], side, ln))
            jobs.append((None if ln == 0 else self.lane_streams[ln], body, ln))
            if body2 is not None:  # (a second job per lane on its own stream)
                jobs.append((self.lane_streams2[ln], body2, ln))
        for st, _, _ in jobs:
            if st is not None:
                st.wait_stream(main)
        res = []
        for st, fn, ln in jobs:
            if st is None:
                r = fn(ln)
            else:
                with torch.cuda.stream(st):
                    r = fn(ln)
            if fn is body:
                res.append(r)
        for st, _, _ in jobs:
            if st is not None:
                main.wait_stream(st)
        return res

    def _rest(self, ln, cur):
        pts, g = self.bufs[ln][cur]
        return hregnet_forward(self.P, self.src[ln], self.dst[ln], self.use_weights, l1=g,
                               pts=pts, v2=self.v2, sub_batch=self.sub_batch)

    def _front_into(self, ln, cur):
        """Lane ln's feature extraction from stage-1 set cur, copied into fe[cur][ln]."""
        pts, g = self.bufs[ln][cur]
        fe = hregnet_front(self.P, self.src[ln], self.dst[ln], self.use_weights, l1=g, pts=pts)
        # the 12 tensors in one launch (hreg_copy_many) instead of 12 copy nodes per lane and round
        dst = self.fe[cur][ln]
        copy_many([dst[k] for k in FRONT_KEYS], [fe[k] for k in FRONT_KEYS])

    def prime(self):
        """Front streaming: run the next round's feature extraction (and the stage 1 of the
        round after) now, so that the next streaming call of whole rounds replays g_fs only.
        A no-op without front streaming or when already primed."""
        if not self.fs or self.fready is not None:
            return
        if self.ready is not None:
            cur = self.ready
        else:
            self.g_first.replay()
            cur = 0
        self.g_prime[cur].replay()
        self.ready = None
        self.fready = 1 - cur

    def load(self, src, dst, lane: int = 0):
        self.src[lane].copy_(src)
        self.dst[lane].copy_(dst)
        self.ready = None  # a streamed stage 1 was made from the old contents
        self.fready = None  # (and streamed fronts)

    def check(self):
        """Raise if a replayed multi-workgroup FPS flagged a poll timeout (synchronous
        when the graphs hold such launches -- Model_V2's clouds above 16384 points -- and a
        no-op otherwise).  run() and run_forwards() call it after their replays."""
        if self.status_check:
            check_device_status(force=True)

    def _partial(self, r: int):
        """Graphs for a partial round of r < lanes forwards (captured on first use):
        first = stage 1 of lanes < r; steps[cur] = the rest of every lane's batch with stage
        1 of the next batch on lanes < r only; lasts[cur] = the rest of lanes < r; streaming
        (batched stage 1 only): psteps[cur] = the rest of lanes < r with the next round's
        batched stage 1 of every lane."""
        if r in self._part:
            return self._part[r]
        torch.cuda.synchronize()
        g = {"first": torch.cuda.CUDAGraph(), "steps": [], "souts": [], "lasts": [],
             "louts": [], "psteps": [], "pouts": []}
        with capture.graph(g["first"], pool=self.pool):
            self._first_stage1(lanes=r)  # (batched: every lane's stage 1, the extra lanes unused)
        for cur in (0, 1):
            variants = [("steps", "souts", self._side_kw(1 - cur, side_lanes=r)),
                        ("lasts", "louts", {"lanes": r})]
            if self.bs1:
                variants.append(("psteps", "pouts", {"lanes": r, **self._side_kw(1 - cur)}))
            for gk, ok, kw in variants:
                gr = torch.cuda.CUDAGraph()
                with capture.graph(gr, pool=self.pool):
                    out = self._fork(lambda ln: self._rest(ln, cur), **kw)
                g[gk].append(gr)
                g[ok].append(out)
        torch.cuda.synchronize()
        self._part[r] = g
        return g

    def prepare(self, n: int):
        """Capture ahead what run_forwards(n) needs (the partial-round graphs)."""
        if n % self.lanes:
            self._partial(n % self.lanes)

    def _finish(self, outs):
        """Per-lane outputs of one replay (Model_V2: the host-RNG prime shuffles of this
        round, drawn after its replay as the reference draws them per forward)."""
        return [model_v2_finish(o, self.sub_batch) for o in outs] if self.v2 else list(outs)

    def run_forwards(self, n: int, stream: bool = False):
        """n forwards in all: full rounds of every lane, then (n % lanes) forwards on the
        first lanes (a partial round: lanes < n % lanes run one forward more).  Returns the
        last forward's output of every lane (views into graph-owned memory; None for a lane
        that ran none).

        stream=True (batched stage 1 only, clouds <= 16384 points): the executor as a
        continuous stream -- the last replay also runs the NEXT round's stage 1 (level-1
        FPS + spatial index + kNN of every lane's batch) beside its forwards, and the next
        call starts from it instead of running stage 1 alone first.  Every call still runs
        exactly one batched stage 1 per round; load() discards a streamed stage 1."""
        if n <= 0:
            return None
        q, r = divmod(n, self.lanes)
        streaming = stream and self.bs1
        if self.fready is not None:
            if streaming and r == 0:
                cur = self.fready
                full = [None] * self.lanes
                for _ in range(q):
                    self.g_fs[cur].replay()
                    full = self._finish(self.outs_fs[cur])
                    cur = 1 - cur
                self.fready = cur
                self.check()
                return full
            # (static inputs: the pending fronts would repeat the forwards this call runs;
            # their stage 1 -- the same batches' -- is the next round's)
            self.ready, self.fready = self.fready, None
        part = self._partial(r) if r else None
        if self.ready is not None:
            cur = self.ready
        else:
            (self.g_first if q or part is None else part["first"]).replay()
            cur = 0
        self.ready = None
        full = [None] * self.lanes
        for i in range(q):
            if i == q - 1 and r:      # stage 1 of the partial round's lanes next
                g, o = part["steps"][cur], part["souts"][cur]
            elif i == q - 1 and not streaming:
                g, o = self.g_last[cur], self.outs_last[cur]
            else:
                g, o = self.g_step[cur], self.outs[cur]
            g.replay()
            full = self._finish(o)
            cur = 1 - cur
        if r:
            g, o = (part["psteps"][cur], part["pouts"][cur]) if streaming else \
                   (part["lasts"][cur], part["louts"][cur])
            g.replay()
            full = self._finish(o) + full[r:]
            cur = 1 - cur
        if streaming:
            self.ready = cur
        self.check()
        return full

    def run(self, steps: int):
        """Runs `steps` rounds; a round is one complete forward of every lane's static
        batch.  Returns the last round's output dict (lanes == 1) or the list of
        per-lane dicts (views into graph-owned memory, valid until the next run)."""
        if steps <= 0:
            return None
        out = self.run_forwards(steps * self.lanes)
        return out[0] if self.lanes == 1 else out
