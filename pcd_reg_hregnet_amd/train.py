"""Training-step building blocks on the HIP library.

The reference trains HRegNet with train-mode BatchNorm after every 1x1 conv
(models/HRegNet/layers.py:115-130, 183-198, 246-268, 417-431), Adam
(train/train_reg_v0.py:246-247) and DDP over NCCL (config 4: one bucketed all-reduce
of the 2,467,846 fp32 gradients per step).  Here:

* ``conv_bn_act``: autograd function for Conv(1x1, rows x channels) + BatchNorm
  (batch statistics, running-stat update) + optional ReLU.  Forward: hreg_gemm
  (fp32 MFMA, bias as the epilogue shift), hreg_bn_stats, hreg_bn_apply.
  Backward: hreg_bn_backward (dgamma, dbeta, dy), hreg_gemm_tn (dW = dy^T x),
  hreg_col_sum (dbias), hreg_gemm with W^T (dx = dy W).
* ``Adam``: torch.optim.Adam's update (weight decay 0) as one kernel per parameter.
* ``GradBucket``: every gradient in one flat fp32 buffer, averaged over ranks with a
  single ``all_reduce`` (RCCL over xGMI on the GPU; gloo in the CPU tests).

torch is plumbing here (autograd bookkeeping, allocation, torch.distributed); every
arithmetic op runs in the HIP library, which must be present (no CPU fallback).
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist

from . import _lib, engine, switches

BN_MOMENTUM = 0.1  # nn.BatchNorm default
BN_EPS = 1e-5
# conv products (forward and input-gradient GEMMs) on hreg_gemm6: fp32-accurate bf16x6
# products on the bf16 matrix cores (engine.B6_GEMM) instead of the f32 MFMA
# for outputs at least TRAIN_B6_MIN_N wide (hreg_gemm6 has 128 x 128 tiles only: narrower
# outputs stay on hreg_gemm's 256 x 32 / 256 x 64 tiles).  Off: the step gains 1-3 % (noise
# level, tools/train_ab.sh) and the reference-gradient test's d/d dst_sigmas_3 error moves
# to 1.16x its bar.
TRAIN_B6 = switches.flag("TRAIN_B6", False)
TRAIN_B6_MIN_N = 128


def _stream():
    return _lib.stream_handle()


def _ws(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


def col_reduce_ws(R: int, C: int, device) -> torch.Tensor:
    return _ws(_lib.load().hreg_col_reduce_ws_bytes(R, C), device)


def bn_stats(y: torch.Tensor, eps: float = BN_EPS):
    """per-channel (mean, invstd, unbiased var) of y [R][C] (batch statistics)."""
    R, C = y.shape
    dev = y.device
    mean = torch.empty(C, device=dev)
    invstd = torch.empty(C, device=dev)
    var = torch.empty(C, device=dev)
    _lib.call("hreg_bn_stats", y, R, C, float(eps), col_reduce_ws(R, C, dev), mean, invstd, var,
              _stream())
    return mean, invstd, var


def gemm_tn(A: torch.Tensor, B: torch.Tensor, into: torch.Tensor | None = None) -> torch.Tensor:
    """A [R][N], B [R][K] -> A^T B [N][K] (fp32 MFMA, deterministic split-R reduction);
    into: added to that [N][K] tensor instead (returned)."""
    R, N = A.shape
    K = B.shape[1]
    out = into if into is not None else torch.empty(N, K, device=A.device)
    ws = _ws(_lib.load().hreg_gemm_tn_ws_bytes(R, N, K), A.device)
    _lib.call("hreg_gemm_tn", A, A.stride(0), B, B.stride(0), R, N, K,
              1.0 if into is not None else 0.0, ws, out, _stream())
    return out


def transpose(x: torch.Tensor) -> torch.Tensor:
    R, C = x.shape
    out = torch.empty(C, R, device=x.device)
    _lib.call("hreg_transpose", x, R, C, out, _stream())
    return out


def col_sum(x: torch.Tensor, into: torch.Tensor | None = None) -> torch.Tensor:
    """column sums of x [R][C]; into: added to that tensor instead (returned)"""
    R, C = x.shape
    out = into if into is not None else torch.empty(C, device=x.device)
    _lib.call("hreg_col_sum", x, R, C, col_reduce_ws(R, C, x.device), out,
              1 if into is not None else 0, _stream())
    return out


DIRECT_GRAD = True  # (A/B switch: False returns every parameter gradient to autograd)
# Direct gradients are on only between GradBucket.attach and GradBucket.collect (the
# trainers' steps) or inside direct_gradients(): outside them every parameter gradient goes
# back to autograd, so torch.autograd.grad / backward(inputs=...) and gradient hooks see the
# usual behaviour.
_DIRECT_ON = False


@contextlib.contextmanager
def direct_gradients():
    """backwards run inside add parameter gradients into existing .grad tensors in place"""
    global _DIRECT_ON
    old = _DIRECT_ON
    _DIRECT_ON = True
    try:
        yield
    finally:
        _DIRECT_ON = old

# Two-stream training step (train_graph.hregnet_train_forward(concurrent=True)): the src and
# dst feature extractions run on two streams, and so do their backwards.  A layer records the
# side it ran on; side 1 adds its parameter gradients into the gradient bucket's second buffer
# (GradBucket(sides=2): p._grad_side1), side 0 into p.grad, so the two streams never add into
# the same memory; GradBucket.collect adds the second buffer into the first (g_src + g_dst:
# the same fp32 sum as autograd's serial accumulation, which is commutative for two terms).
# The dst side's BN running-statistics updates are deferred (DEFERRED_RUNNING) and applied
# after the src side's, in the reference's order.
_SIDE = 0
DEFERRED_RUNNING: list | None = None  # when a list: (mean, var, running_mean, running_var, momentum)


@contextlib.contextmanager
def side(s: int, defer_running: bool = False):
    """layers built inside run as side s (gradient bucket s); defer_running: their BN
    running-statistics updates are queued in the yielded list instead of applied"""
    global _SIDE, DEFERRED_RUNNING
    old = (_SIDE, DEFERRED_RUNNING)
    queued = [] if defer_running else None
    _SIDE, DEFERRED_RUNNING = s, queued
    try:
        yield queued
    finally:
        _SIDE, DEFERRED_RUNNING = old


def apply_running(updates) -> None:
    """hreg_bn_running_update for queued (mean, var_unbiased, running_mean, running_var,
    momentum) entries, in order, on the current stream"""
    for mean, var, rm, rv, momentum in updates:
        _lib.call("hreg_bn_running_update", mean, var, mean.shape[0], float(momentum), rm, rv, _stream())


def _grad_slot(p, side: int = 0):
    """The buffer the backward of a side-`side` layer may add p's gradient to in place
    (autograd's own accumulation into an existing .grad: the flat gradient bucket is
    attached and zeroed every step; side 1: the bucket's second buffer), else None (return
    the gradient to autograd)"""
    if p is None or not p.requires_grad or not (DIRECT_GRAD and _DIRECT_ON):
        return None
    g = p.grad if side == 0 else getattr(p, "_grad_side1", None)
    if g is None or not g.is_contiguous() or g.dtype != torch.float32:
        return None
    return g


_CONST = {}


def _const(value: float, n: int, device) -> torch.Tensor:
    """Cached constant vectors (the unit scale / zero shift of a plain GEMM epilogue)."""
    key = (value, n, str(device))
    t = _CONST.get(key)
    if t is None:
        t = _CONST[key] = torch.full((n,), value, dtype=torch.float32, device=device)
    return t


def _plain_gemm(x: torch.Tensor, W: torch.Tensor, shift: torch.Tensor | None) -> torch.Tensor:
    """x [R][K] @ W[N][K]^T (+ shift) on hreg_gemm (no activation)."""
    R, K = x.shape
    N = W.shape[0]
    ones = _const(1.0, N, x.device)
    sh = shift if shift is not None else _const(0.0, N, x.device)
    lin = engine.Lin(W.contiguous(), ones, sh.contiguous(), relu=False)
    return engine.gemm([engine._seg(x, 0, K)], lin, R, b6=TRAIN_B6 and N >= TRAIN_B6_MIN_N)


# conv GEMMs of >= TS_MIN_ROWS rows on hreg_ts_gemm (the tall-skinny kernel: W in LDS, A
# streamed from HBM; the same fp32 sums as hreg_gemm); the input gradient reads W in place.
# (r6: 4096 -- the level-1 / level-2 detector heads' 8192 / 4096 rows join it, and with it the
# fused statistics and the chains: eager step 22.10 -> 21.27 ms, 1024 21.65; r5: 16384)
TS_GEMM = True
TS_MIN_ROWS = 4096


def _conv_gemm(x: torch.Tensor, W: torch.Tensor, shift: torch.Tensor | None,
               w_trans: bool = False) -> torch.Tensor:
    """x [R][K] @ W'^T (+ shift) with W' = W [N][K], or W [K][N] transposed (w_trans)."""
    R, K = x.shape
    N = W.shape[1] if w_trans else W.shape[0]
    lib = _lib.load()
    if (TS_GEMM and R >= TS_MIN_ROWS and x.is_contiguous() and W.is_contiguous()
            and lib.hreg_ts_gemm_supported(R, K, N, 0)):
        out = torch.empty(R, N, device=x.device)
        _lib.call("hreg_ts_gemm", x, K, R, K, W, 1 if w_trans else 0, N, None,
                  None if shift is None else shift.contiguous(), 0, out, N, _stream())
        return out
    return _plain_gemm(x, transpose(W) if w_trans else W, shift)


TS_BN = True  # (A/B switch: the statistics pass fused into hreg_ts_gemm's epilogue)


def _conv_gemm_bn(x, W, shift, eps, momentum, running_mean, running_var):
    """(y, mean, invstd, var_unbiased) from hreg_ts_gemm_bn when the conv takes the tall-skinny
    path (running stats updated there), else None."""
    R, K = x.shape
    N = W.shape[0]
    lib = _lib.load()
    if not (TS_GEMM and TS_BN and R >= TS_MIN_ROWS and x.is_contiguous() and W.is_contiguous()
            and lib.hreg_ts_gemm_supported(R, K, N, 1)):
        return None
    dev = x.device
    y = torch.empty(R, N, device=dev)
    mean, invstd, var = (torch.empty(N, device=dev) for _ in range(3))
    ws = _ws(lib.hreg_ts_gemm_bn_ws_bytes(R, K, N), dev)
    _lib.call("hreg_ts_gemm_bn", x, K, R, K, W, 0, N, None if shift is None else shift.contiguous(),
              y, N, float(eps), float(momentum), ws, mean, invstd, var, running_mean, running_var,
              _stream())
    return y, mean, invstd, var


class _ConvBNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, bias, gamma, beta, running_mean, running_var, relu, momentum, eps,
                wparam=None):
        R = x.shape[0]
        defer = DEFERRED_RUNNING is not None and running_mean is not None
        rm, rv = (None, None) if defer else (running_mean, running_var)
        fused = _conv_gemm_bn(x, W, bias, eps, momentum, rm, rv)
        if fused is not None:
            y, mean, invstd, var = fused  # statistics (+ running update) in the GEMM's epilogue
        else:
            y = _conv_gemm(x, W, bias)
            mean, invstd, var = bn_stats(y, eps)
            if rm is not None:
                _lib.call("hreg_bn_running_update", mean, var, y.shape[1], float(momentum),
                          rm, rv, _stream())
        if defer:
            DEFERRED_RUNNING.append((mean, var, running_mean, running_var, momentum))
        ctx.side = _SIDE
        C = y.shape[1]
        out = torch.empty_like(y)
        _lib.call("hreg_bn_apply", y, R, C, mean, invstd, gamma, beta, 1 if relu else 0, out,
                  _stream())
        ctx.save_for_backward(x, W, y, mean, invstd, gamma, beta)
        ctx.relu = relu
        ctx.has_bias = bias is not None
        # the parameter objects whose .grad the backward may add to directly (W is usually
        # a [N][K] view of the conv weight; bias / gamma / beta are the parameters)
        ctx.params = (wparam, bias, gamma, beta)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, W, y, mean, invstd, gamma, beta = ctx.saved_tensors
        dout = dout.contiguous()
        R, C = y.shape
        dev = y.device
        dy = torch.empty_like(y)
        # parameter gradients straight into an existing .grad (the gradient bucket): the
        # same fp32 sums autograd's accumulation would make (g_src + g_dst, added to the
        # zeroed .grad), without its two elementwise additions per parameter and use
        wp, bp, gp, btp = ctx.params
        gw = _grad_slot(wp, ctx.side) if ctx.needs_input_grad[1] else None
        gb = _grad_slot(bp, ctx.side) if ctx.has_bias and ctx.needs_input_grad[2] else None
        gg, gbt = _grad_slot(gp, ctx.side), _grad_slot(btp, ctx.side)
        acc = gg is not None and gbt is not None and ctx.needs_input_grad[3] and ctx.needs_input_grad[4]
        dgamma = gg if acc else torch.empty(C, device=dev)
        dbeta = gbt if acc else torch.empty(C, device=dev)
        # the ReLU mask is recomputed from y (bit-identical to bn_apply's): out is not read
        _lib.call("hreg_bn_backward", dout, None, y, R, C, mean, invstd, gamma, beta,
                  1 if ctx.relu else 0, col_reduce_ws(R, C, dev), dy, dgamma, dbeta,
                  1 if acc else 0, _stream())
        dW = None
        if ctx.needs_input_grad[1]:
            if gw is not None:
                gemm_tn(dy, x, into=gw.view(W.shape))
            else:
                dW = gemm_tn(dy, x)
        dbias = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            if gb is not None:
                col_sum(dy, into=gb)
            else:
                dbias = col_sum(dy)
        dx = _conv_gemm(dy, W, None, w_trans=True) if ctx.needs_input_grad[0] else None
        if acc:
            dgamma = dbeta = None
        return dx, dW, dbias, dgamma, dbeta, None, None, None, None, None, None


def conv_bn_act(x, W, bias, gamma, beta, running_mean=None, running_var=None, relu=True,
                momentum=BN_MOMENTUM, eps=BN_EPS, wparam=None):
    """Train-mode Conv1x1 + BatchNorm + [ReLU] over rows: x [R][K] (K % 4 == 0),
    W [N][K] -> [R][N].  Matches nn.Conv1d/Conv2d(k=1) + nn.BatchNorm*d(train) + nn.ReLU
    on the same rows (every position of the batch is a row).  wparam: the parameter W is a
    view of (its .grad, like bias' / gamma's / beta's, is added to in place when present)."""
    return _ConvBNAct.apply(x.contiguous(), W, bias, gamma, beta, running_mean, running_var,
                            relu, momentum, eps, wparam if wparam is not None else W)


def tail_fusable(R: int, k: int, C1: int, Ca: int, N: int) -> bool:
    """_TailConvBNAct's kernels take this shape (else the concatenation path runs)"""
    K = 2 * C1 + Ca
    return (TS_GEMM and TS_BN and R >= TS_MIN_ROWS and R % k == 0 and C1 % 64 == 0 and Ca % 64 == 0
            and bool(_lib.load().hreg_ts_gemm_supported(R, K, N, 1)))


def _tail_forward(x1, att, W, bias, running_mean, running_var, k, momentum, eps):
    """The tail conv's pre-BN output and statistics -> (y, mean, invstd, x2, arg)"""
    R, C1 = x1.shape
    Ca = att.shape[1]
    G = R // k
    N = W.shape[0]
    dev = x1.device
    st = _stream()
    x2 = torch.empty(G, C1, device=dev)
    arg = torch.empty(G, C1, dtype=torch.int32, device=dev)
    _lib.call("hreg_group_max_arg", x1, C1, G, k, C1, x2, C1, arg, st)
    defer = DEFERRED_RUNNING is not None and running_mean is not None
    rm, rv = (None, None) if defer else (running_mean, running_var)
    y = torch.empty(R, N, device=dev)
    mean, invstd, var = (torch.empty(N, device=dev) for _ in range(3))
    ws = _ws(_lib.load().hreg_ts_gemm_bn_ws_bytes(R, 2 * C1 + Ca, N), dev)
    _lib.call("hreg_ts_gemm_bn_tail", x2, k, x1, C1, att, Ca, R, W.contiguous(), N,
              None if bias is None else bias.contiguous(), y, N, float(eps), float(momentum), ws, mean, invstd,
              var, rm, rv, st)
    if defer:
        DEFERRED_RUNNING.append((mean, var, running_mean, running_var, momentum))
    return y, mean, invstd, x2, arg


def _tail_backward(ctx, dy, x1, att, x2, arg, W, need_x1, need_att, need_W, need_b):
    """The tail conv's backward from dL/dy (pre-BN) -> (dx1, datt, dW, dbias); W / bias
    gradients added into their .grad buffers in place when the trainers attach them"""
    R, N = dy.shape
    C1, Ca = x1.shape[1], att.shape[1]
    k = ctx.k
    G = R // k
    K = 2 * C1 + Ca
    dev = dy.device
    st = _stream()
    wp, bp = ctx.params[:2]
    gw = _grad_slot(wp, ctx.side) if need_W else None
    gb = _grad_slot(bp, ctx.side) if ctx.has_bias and need_b else None
    dW = None
    if need_W:
        out = gw.view(W.shape) if gw is not None else torch.empty(N, K, device=dev)
        ws = _ws(_lib.load().hreg_gemm_tn_ws_bytes(R, N, K), dev)
        _lib.call("hreg_gemm_tn_tail", dy, N, x2, k, x1, C1, att, Ca, R, N, 1.0 if gw is not None else 0.0,
                  ws, out, st)
        if gw is None:
            dW = out
    dbias = None
    if ctx.has_bias and need_b:
        if gb is not None:
            col_sum(dy, into=gb)
        else:
            dbias = col_sum(dy)
    dx1 = datt = None
    if need_x1 or need_att:
        # the [R][K] input gradient (desc_tail's backward from here): its x1 and att_map blocks
        # written straight into their own gradients when the tall-skinny GEMM takes the shape
        if (TS_GEMM and R >= TS_MIN_ROWS and C1 % 32 == 0 and W.is_contiguous() and
                _lib.load().hreg_ts_gemm_supported(R, N, K, 0)):
            drep = torch.empty(R, C1, device=dev)
            dx1 = torch.empty(R, C1, device=dev)
            datt = torch.empty(R, Ca, device=dev)
            _lib.call("hreg_ts_gemm_split_out", dy, N, R, N, W, 1, K, drep, C1, C1, dx1, C1, 2 * C1, datt, Ca, st)
        else:
            dcat = _conv_gemm(dy, W, None, w_trans=True)
            drep, datt = dcat, dcat[:, 2 * C1:]
            dx1 = torch.empty(R, C1, device=dev)
            _lib.call("hreg_copy_rows", dcat[:, C1:], K, 1, R, C1, dx1, C1, 0, st)
        if need_x1:
            dx2 = torch.empty(G, C1, device=dev)
            _lib.call("hreg_group_sum", drep, drep.stride(0), G, k, C1, dx2, C1, 0, st)
            _lib.call("hreg_group_max_bwd", dx2, C1, arg, G, k, C1, dx1, C1, 1, st)
        else:
            dx1 = None
        if not need_att:
            datt = None
    return dx1, datt, dW, dbias


class _TailConvBNAct(torch.autograd.Function):
    """The descriptor's mlp1 (Conv1x1 + train-mode BN + ReLU) over cat([x2 repeated over each
    group's k rows, x1, att_map]) (layers.py:202-209) without materialising the concatenation
    (r6): the forward GEMM + statistics (hreg_ts_gemm_bn_tail) and the weight gradient
    (hreg_gemm_tn_tail) read the three blocks in place.  Every kernel computes the concatenation
    path's sums in its order (the same values in the same k / row order), and the input gradients
    are the concatenation path's (the [R][2 C1 + Ca] gradient, its x2 block summed per group and
    sent to the argmax rows), so outputs and gradients are bitwise those of desc_tail +
    conv_bn_act."""

    @staticmethod
    def forward(ctx, x1, att, W, bias, gamma, beta, running_mean, running_var, k, momentum, eps, wparam=None):
        y, mean, invstd, x2, arg = _tail_forward(x1, att, W, bias, running_mean, running_var, k, momentum, eps)
        R, N = y.shape
        out = torch.empty_like(y)
        _lib.call("hreg_bn_apply", y, R, N, mean, invstd, gamma, beta, 1, out, _stream())
        ctx.save_for_backward(x1, att, x2, arg, W, y, mean, invstd, gamma, beta)
        ctx.side = _SIDE
        ctx.k = k
        ctx.has_bias = bias is not None
        ctx.params = (wparam, bias, gamma, beta)
        return out

    @staticmethod
    def backward(ctx, dout):
        x1, att, x2, arg, W, y, mean, invstd, gamma, beta = ctx.saved_tensors
        dout = dout.contiguous()
        R, N = y.shape
        dev = y.device
        gp, btp = ctx.params[2:]
        gg, gbt = _grad_slot(gp, ctx.side), _grad_slot(btp, ctx.side)
        acc = gg is not None and gbt is not None and ctx.needs_input_grad[4] and ctx.needs_input_grad[5]
        dgamma = gg if acc else torch.empty(N, device=dev)
        dbeta = gbt if acc else torch.empty(N, device=dev)
        dy = torch.empty_like(y)
        _lib.call("hreg_bn_backward", dout, None, y, R, N, mean, invstd, gamma, beta, 1,
                  col_reduce_ws(R, N, dev), dy, dgamma, dbeta, 1 if acc else 0, _stream())
        dx1, datt, dW, dbias = _tail_backward(ctx, dy, x1, att, x2, arg, W, *ctx.needs_input_grad[:4])
        if acc:
            dgamma = dbeta = None
        return dx1, datt, dW, dbias, dgamma, dbeta, None, None, None, None, None, None


class _TailConvStats(torch.autograd.Function):
    """_TailConvBNAct without its BN apply: -> (y pre-BN, mean, invstd) for a chain's next conv to
    apply on load (tail_conv_bn_chain)."""

    @staticmethod
    def forward(ctx, x1, att, W, bias, running_mean, running_var, k, momentum, eps, wparam):
        y, mean, invstd, x2, arg = _tail_forward(x1, att, W, bias, running_mean, running_var, k, momentum, eps)
        ctx.save_for_backward(x1, att, x2, arg, W)
        ctx.side = _SIDE
        ctx.k = k
        ctx.has_bias = bias is not None
        ctx.params = (wparam, bias)
        ctx.mark_non_differentiable(mean, invstd)
        return y, mean, invstd

    @staticmethod
    def backward(ctx, dy, _dmean, _dinvstd):
        x1, att, x2, arg, W = ctx.saved_tensors
        dx1, datt, dW, dbias = _tail_backward(ctx, dy.contiguous(), x1, att, x2, arg, W, *ctx.needs_input_grad[:4])
        return dx1, datt, dW, dbias, None, None, None, None, None, None


def tail_conv_bn_act(x1, att, k, W, bias, gamma, beta, running_mean=None, running_var=None,
                     momentum=BN_MOMENTUM, eps=BN_EPS, wparam=None):
    """Conv1x1 + train-mode BN + ReLU over cat([max_k x1 repeated over k rows, x1, att]) without
    the concatenation (_TailConvBNAct; the caller checks tail_fusable); W [N][2 C1 + Ca]."""
    return _TailConvBNAct.apply(x1.contiguous(), att.contiguous(), W, bias, gamma, beta, running_mean,
                                running_var, k, momentum, eps, wparam if wparam is not None else W)


def tail_chain_fusable(R: int, k: int, C1: int, Ca: int, widths) -> bool:
    """tail_conv_bn_chain takes the tail conv (widths[0] = its N) and the convs after it"""
    return (CHAIN_FUSED and len(widths) >= 2 and tail_fusable(R, k, C1, Ca, widths[0]) and
            all(w % 4 == 0 for w in widths) and
            all(_lib.load().hreg_ts_gemm_pre_supported(R, widths[i], widths[i + 1]) for i in range(len(widths) - 1)))


def tail_conv_bn_chain(x1, att, k, tail, layers, group_max=False):
    """tail_conv_bn_act followed by conv_bn_act for each of `layers` (conv_bn_chain's tuples),
    the inner activations never written; tail = (W, bias, gamma, beta, running_mean, running_var,
    momentum, eps, wparam); group_max: the max over each group's k rows of the last activation
    instead of the activation (not written either).  Bitwise the layerwise path (the caller checks
    tail_chain_fusable)."""
    W, bias, gamma, beta, rm, rv, momentum, eps, wparam = tail
    y, mean, invstd = _TailConvStats.apply(x1.contiguous(), att.contiguous(), W, bias, rm, rv, k, momentum, eps,
                                           wparam if wparam is not None else W)
    pre = (mean, invstd, gamma, beta)
    for W, bias, gamma, beta, rm, rv, momentum, eps, wparam in layers:
        y, mean, invstd = _ConvStats.apply(y, W, bias, *pre, rm, rv, momentum, eps,
                                           wparam if wparam is not None else W)
        pre = (mean, invstd, gamma, beta)
    return _BNActGroupMax.apply(y, *pre, k) if group_max else _BNAct.apply(y, *pre)


# Chains of Conv + train-mode BN + ReLU layers (nn.Sequential, layers.py:115-130, 183-198) with the
# inner activations never materialised (r6): each conv after the first reads the previous layer's
# pre-BN output and applies that BN + ReLU on load (hreg_ts_gemm_bn_pre forward, hreg_gemm_tn_pre
# weight gradient), and only the chain's last activation is written (_BNAct).  Every kernel
# computes conv_bn_act's values in its order, so outputs and gradients are bitwise its own.
CHAIN_FUSED = switches.flag("CHAIN_FUSED", True)


class _ConvStats(torch.autograd.Function):
    """y = act_prev(x) W^T + bias with this layer's train-mode BN statistics (and running update);
    act_prev = the previous layer's BN + ReLU (pre_* tensors) or the identity (the chain's first
    layer).  -> y (pre-BN), mean, invstd.  The backward returns dL/dx through act_prev: the
    previous layer's BN backward runs here (its dgamma / dbeta into the previous BN's .grad)."""

    @staticmethod
    def forward(ctx, x, W, bias, pre_mean, pre_invstd, pre_gamma, pre_beta, running_mean, running_var,
                momentum, eps, wparam):
        R, K = x.shape
        N = W.shape[0]
        dev = x.device
        st = _stream()
        defer = DEFERRED_RUNNING is not None and running_mean is not None
        rm, rv = (None, None) if defer else (running_mean, running_var)
        y = torch.empty(R, N, device=dev)
        mean, invstd, var = (torch.empty(N, device=dev) for _ in range(3))
        ws = _ws(_lib.load().hreg_ts_gemm_bn_ws_bytes(R, K, N), dev)
        shift = None if bias is None else bias.contiguous()
        if pre_mean is None:
            _lib.call("hreg_ts_gemm_bn", x, K, R, K, W, 0, N, shift, y, N, float(eps), float(momentum), ws,
                      mean, invstd, var, rm, rv, st)
        else:
            _lib.call("hreg_ts_gemm_bn_pre", x, K, R, K, W, N, shift, y, N, float(eps), float(momentum), ws,
                      mean, invstd, var, rm, rv, pre_mean, pre_invstd, pre_gamma, pre_beta, 1, st)
        if defer:
            DEFERRED_RUNNING.append((mean, var, running_mean, running_var, momentum))
        ctx.save_for_backward(x, W, pre_mean, pre_invstd, pre_gamma, pre_beta)
        ctx.side = _SIDE
        ctx.pre = pre_mean is not None
        ctx.has_bias = bias is not None
        ctx.params = (wparam, bias, pre_gamma, pre_beta)
        ctx.mark_non_differentiable(mean, invstd)
        return y, mean, invstd

    @staticmethod
    def backward(ctx, dy, _dmean, _dinvstd):
        x, W, pm, pi, pg, pbt = ctx.saved_tensors
        dy = dy.contiguous()
        R, N = dy.shape
        K = x.shape[1]
        dev = dy.device
        st = _stream()
        wp, bp, gp, btp = ctx.params
        gw = _grad_slot(wp, ctx.side) if ctx.needs_input_grad[1] else None
        gb = _grad_slot(bp, ctx.side) if ctx.has_bias and ctx.needs_input_grad[2] else None
        dW = None
        if ctx.needs_input_grad[1]:
            if ctx.pre:
                out = gw.view(W.shape) if gw is not None else torch.empty(N, K, device=dev)
                ws = _ws(_lib.load().hreg_gemm_tn_ws_bytes(R, N, K), dev)
                _lib.call("hreg_gemm_tn_pre", dy, N, x, K, R, N, K, 1.0 if gw is not None else 0.0, ws, out,
                          pm, pi, pg, pbt, 1, st)
                if gw is None:
                    dW = out
            elif gw is not None:
                gemm_tn(dy, x, into=gw.view(W.shape))
            else:
                dW = gemm_tn(dy, x)
        dbias = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            if gb is not None:
                col_sum(dy, into=gb)
            else:
                dbias = col_sum(dy)
        dx = dgamma = dbeta = None
        if ctx.needs_input_grad[0]:
            dx = _conv_gemm(dy, W, None, w_trans=True)  # d act_prev(x)
            if ctx.pre:
                # the previous layer's BN + ReLU backward (conv_bn_act's, with its ReLU mask from x)
                gg, gbt = _grad_slot(gp, ctx.side), _grad_slot(btp, ctx.side)
                acc = gg is not None and gbt is not None and ctx.needs_input_grad[5] and ctx.needs_input_grad[6]
                dgamma = gg if acc else torch.empty(K, device=dev)
                dbeta = gbt if acc else torch.empty(K, device=dev)
                dxy = torch.empty_like(x)
                _lib.call("hreg_bn_backward", dx, None, x, R, K, pm, pi, pg, pbt, 1, col_reduce_ws(R, K, dev), dxy,
                          dgamma, dbeta, 1 if acc else 0, st)
                dx = dxy
                if acc:
                    dgamma = dbeta = None
        return dx, dW, dbias, None, None, dgamma, dbeta, None, None, None, None, None


class _BNAct(torch.autograd.Function):
    """out = ReLU(BN(y)) with the statistics _ConvStats made (the chain's last activation)"""

    @staticmethod
    def forward(ctx, y, mean, invstd, gamma, beta):
        R, C = y.shape
        out = torch.empty_like(y)
        _lib.call("hreg_bn_apply", y, R, C, mean, invstd, gamma, beta, 1, out, _stream())
        ctx.save_for_backward(y, mean, invstd, gamma, beta)
        ctx.side = _SIDE
        ctx.params = (gamma, beta)
        return out

    @staticmethod
    def backward(ctx, dout):
        y, mean, invstd, gamma, beta = ctx.saved_tensors
        dout = dout.contiguous()
        R, C = y.shape
        dev = y.device
        gg, gbt = _grad_slot(ctx.params[0], ctx.side), _grad_slot(ctx.params[1], ctx.side)
        acc = gg is not None and gbt is not None and ctx.needs_input_grad[3] and ctx.needs_input_grad[4]
        dgamma = gg if acc else torch.empty(C, device=dev)
        dbeta = gbt if acc else torch.empty(C, device=dev)
        dy = torch.empty_like(y)
        _lib.call("hreg_bn_backward", dout, None, y, R, C, mean, invstd, gamma, beta, 1, col_reduce_ws(R, C, dev), dy,
                  dgamma, dbeta, 1 if acc else 0, _stream())
        if acc:
            dgamma = dbeta = None
        return dy, None, None, dgamma, dbeta


class _BNActGroupMax(torch.autograd.Function):
    """d = max over each group's k rows of ReLU(BN(y)) with the statistics _ConvStats made: the
    chain's last activation never written either (the descriptor's k-max, layers.py:208-209)"""

    @staticmethod
    def forward(ctx, y, mean, invstd, gamma, beta, k):
        R, C = y.shape
        G = R // k
        d = torch.empty(G, C, device=y.device)
        arg = torch.empty(G, C, dtype=torch.int32, device=y.device)
        _lib.call("hreg_group_max_arg_pre", y, C, G, k, C, d, C, arg, mean, invstd, gamma, beta, _stream())
        ctx.save_for_backward(y, mean, invstd, gamma, beta, arg)
        ctx.side = _SIDE
        ctx.k = k
        ctx.params = (gamma, beta)
        return d

    @staticmethod
    def backward(ctx, dd):
        y, mean, invstd, gamma, beta, arg = ctx.saved_tensors
        dd = dd.contiguous()
        R, C = y.shape
        dev = y.device
        st = _stream()
        dout = torch.empty_like(y)  # (group_max's backward: dd at each group's argument rows)
        _lib.call("hreg_group_max_bwd", dd, C, arg, R // ctx.k, ctx.k, C, dout, C, 0, st)
        gg, gbt = _grad_slot(ctx.params[0], ctx.side), _grad_slot(ctx.params[1], ctx.side)
        acc = gg is not None and gbt is not None and ctx.needs_input_grad[3] and ctx.needs_input_grad[4]
        dgamma = gg if acc else torch.empty(C, device=dev)
        dbeta = gbt if acc else torch.empty(C, device=dev)
        dy = torch.empty_like(y)
        _lib.call("hreg_bn_backward", dout, None, y, R, C, mean, invstd, gamma, beta, 1, col_reduce_ws(R, C, dev), dy,
                  dgamma, dbeta, 1 if acc else 0, st)
        if acc:
            dgamma = dbeta = None
        return dy, None, None, dgamma, dbeta, None


def chain_fusable(R: int, widths) -> bool:
    """conv_bn_chain takes a chain of R rows and channel widths [K0, N0, N1, ...]"""
    if not (CHAIN_FUSED and TS_GEMM and TS_BN and R >= TS_MIN_ROWS and len(widths) >= 3):
        return False
    lib = _lib.load()
    return (bool(lib.hreg_ts_gemm_supported(R, widths[0], widths[1], 1)) and
            all(w % 4 == 0 for w in widths) and
            all(lib.hreg_ts_gemm_pre_supported(R, widths[i], widths[i + 1]) for i in range(1, len(widths) - 1)))


def _chain_pre(x, layers):
    """the chain up to its last layer's pre-BN output -> (y, (mean, invstd, gamma, beta))"""
    pre = (None, None, None, None)
    y = x.contiguous()
    for W, bias, gamma, beta, rm, rv, momentum, eps, wparam in layers:
        y, mean, invstd = _ConvStats.apply(y, W, bias, *pre, rm, rv, momentum, eps,
                                           wparam if wparam is not None else W)
        pre = (mean, invstd, gamma, beta)
    return y, pre


def conv_bn_chain(x, layers):
    """Conv1x1 + train-mode BN + ReLU for each (W [N][K], bias, gamma, beta, running_mean,
    running_var, momentum, eps, wparam) in order, over rows x [R][K0]; the inner activations are
    never written (the caller checks chain_fusable).  Bitwise the conv_bn_act sequence."""
    y, pre = _chain_pre(x, layers)
    return _BNAct.apply(y, *pre)


class _BNActAttention(torch.autograd.Function):
    """The detector's attention (train_graph.attention with vals = logits, layers.py:150-159)
    over ReLU(BN(y)) with the statistics _ConvStats made: the detector's last activation never
    written.  -> (kp [G][3], vmap [R][C], vsum [G][C]); its backward runs the BN backward."""

    @staticmethod
    def forward(ctx, y, mean, invstd, gamma, beta, kx, k):
        R, C = y.shape
        G = R // k
        dev = y.device
        a = torch.empty(R, device=dev)
        amax = torch.empty(R, dtype=torch.int32, device=dev)
        kp = torch.empty(G, 3, device=dev)
        vmap = torch.empty(R, C, device=dev)
        vsum = torch.empty(G, C, device=dev)
        _lib.call("hreg_attention_fwd_pre", y, C, C, mean, invstd, gamma, beta, kx, G, k, a, amax, kp, vmap, C,
                  vsum, C, _stream())
        ctx.save_for_backward(y, mean, invstd, gamma, beta, kx, a, amax)
        ctx.side = _SIDE
        ctx.k = k
        ctx.params = (gamma, beta)
        ctx.set_materialize_grads(False)
        return kp, vmap, vsum

    @staticmethod
    def backward(ctx, dkp, dvmap, dvsum):
        y, mean, invstd, gamma, beta, kx, a, amax = ctx.saved_tensors
        k = ctx.k
        R, C = y.shape
        G = R // k
        dev = y.device
        st = _stream()
        dkp = dkp.contiguous() if dkp is not None else None
        lddm = C
        if dvmap is not None:
            if not (dvmap.dim() == 2 and dvmap.stride(1) == 1 and dvmap.stride(0) >= C):
                dvmap = dvmap.contiguous()
            lddm = dvmap.stride(0)
        dvsum = dvsum.contiguous() if dvsum is not None else None
        dact = torch.empty(R, C, device=dev)
        dkx = torch.empty(R, 3, device=dev) if (dkp is not None and ctx.needs_input_grad[5]) else None
        _lib.call("hreg_attention_bwd_pre", y, C, C, mean, invstd, gamma, beta, kx, G, k, a, amax, dkp, dvmap, lddm,
                  dvsum, C, dact, C, dkx, st)
        gg, gbt = _grad_slot(ctx.params[0], ctx.side), _grad_slot(ctx.params[1], ctx.side)
        acc = gg is not None and gbt is not None and ctx.needs_input_grad[3] and ctx.needs_input_grad[4]
        dgamma = gg if acc else torch.empty(C, device=dev)
        dbeta = gbt if acc else torch.empty(C, device=dev)
        dy = torch.empty_like(y)
        _lib.call("hreg_bn_backward", dact, None, y, R, C, mean, invstd, gamma, beta, 1, col_reduce_ws(R, C, dev), dy,
                  dgamma, dbeta, 1 if acc else 0, st)
        if acc:
            dgamma = dbeta = None
        return dy, None, None, dgamma, dbeta, dkx, None


def conv_bn_chain_attention(x, layers, k, kx):
    """conv_bn_chain followed by the detector's attention over its activation (vals = logits,
    want_map, want_sum), the activation never written -> (kp, vmap, vsum); bitwise
    conv_bn_chain + train_graph.attention (the caller checks chain_fusable)"""
    y, pre = _chain_pre(x, layers)
    return _BNActAttention.apply(y, *pre, kx.contiguous(), k)


class ConvBNAct(torch.nn.Module):
    """Parameters of one 1x1 conv + BatchNorm (+ ReLU) layer, reference naming:
    ``conv.weight [N][K(,1,1)]``, ``conv.bias``, ``bn.weight/bias/running_*``."""

    def __init__(self, K: int, N: int, bias: bool = False, relu: bool = True):
        super().__init__()
        self.W = torch.nn.Parameter(torch.empty(N, K))
        self.bias = torch.nn.Parameter(torch.zeros(N)) if bias else None
        self.gamma = torch.nn.Parameter(torch.ones(N))
        self.beta = torch.nn.Parameter(torch.zeros(N))
        self.register_buffer("running_mean", torch.zeros(N))
        self.register_buffer("running_var", torch.ones(N))
        self.relu = relu
        torch.nn.init.kaiming_uniform_(self.W, a=5 ** 0.5)

    def forward(self, x):
        if not self.training:
            raise NotImplementedError("eval mode runs through engine (folded BN)")
        return conv_bn_act(x, self.W, self.bias, self.gamma, self.beta, self.running_mean,
                           self.running_var, self.relu)


class Adam:
    """torch.optim.Adam (lr, betas, eps; weight decay 0) on the HIP library."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        self.params = [p for p in params if p.requires_grad]
        self.lr, self.betas, self.eps = lr, betas, eps
        self.state = [(torch.zeros_like(p), torch.zeros_like(p)) for p in self.params]
        self.step_count = 0

    def zero_grad(self):
        for p in self.params:
            p.grad = None

    @torch.no_grad()
    def step(self):
        self.step_count += 1
        for p, (m, v) in zip(self.params, self.state):
            if p.grad is None:
                continue
            _lib.call("hreg_adam_step", p, p.grad.contiguous(), m, v, p.numel(), float(self.lr),
                      float(self.betas[0]), float(self.betas[1]), float(self.eps),
                      self.step_count, _stream())


FLAT_ALIGN = 64  # floats: every tensor of a flat buffer starts on a 256-byte boundary


def flat_offsets(params):
    """Offsets of each tensor in a flat buffer (aligned for the kernels' dwordx4 loads)
    and the padded total."""
    offs, off = [], 0
    for p in params:
        offs.append(off)
        off += -(-p.numel() // FLAT_ALIGN) * FLAT_ALIGN
    return offs, off


class GradBucket:
    """All of a model's gradients in one flat fp32 buffer, averaged over the ranks with a
    single all_reduce (9.87 MB for HRegNet -- one bucket, so one ring
    pass over xGMI per step instead of one collective per tensor).  After ``attach``
    every parameter's .grad is a view into the buffer, so the backward writes straight
    into it."""

    def __init__(self, params, sides: int = 1):
        self.params = [p for p in params if p.requires_grad]
        offs, n = flat_offsets(self.params)
        dev = self.params[0].device if self.params else torch.device("cpu")
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.views = [self.flat[o:o + p.numel()].view_as(p) for p, o in zip(self.params, offs)]
        # sides = 2: a second buffer for the gradients of side-1 layers (train.side), so the
        # two streams of the two-stream step never add into the same memory
        self.flat1 = torch.zeros(n, dtype=torch.float32, device=dev) if sides == 2 else None
        self.views1 = ([self.flat1[o:o + p.numel()].view_as(p) for p, o in zip(self.params, offs)]
                       if sides == 2 else None)

    def attach(self):
        """Point every .grad at its slice (zeroed); sides = 2: also p._grad_side1.  Turns the
        direct parameter gradients on until ``collect``."""
        global _DIRECT_ON
        _DIRECT_ON = True
        self.flat.zero_()
        for p, v in zip(self.params, self.views):
            p.grad = v
        if self.flat1 is not None:
            self.flat1.zero_()
            for p, v in zip(self.params, self.views1):
                p._grad_side1 = v

    @staticmethod
    def direct_off():
        """Turn the direct parameter gradients off (idempotent).  The trainers call it in a
        ``finally`` after ``attach``, so a forward / backward that raises between ``attach``
        and ``collect`` cannot leave them on for later autograd calls."""
        global _DIRECT_ON
        _DIRECT_ON = False

    def collect(self, two_sides: bool = False):
        """Copy gradients that autograd allocated separately into the buffer; two_sides (after a
        two-stream step): add the second buffer (side-1 gradients) into it.  Turns the direct
        parameter gradients off."""
        global _DIRECT_ON
        _DIRECT_ON = False
        for p, v in zip(self.params, self.views):
            if p.grad is None:
                v.zero_()
            elif p.grad.data_ptr() != v.data_ptr():
                v.copy_(p.grad)
                p.grad = v
        if two_sides:
            if self.flat1 is None:
                raise RuntimeError("GradBucket: two_sides needs sides=2")
            _lib.call("hreg_add_into", self.flat1, self.flat, self.flat.numel(), _stream())

    def all_reduce_mean(self, group=None, force: bool = False):
        """SUM over the ranks, then / world.  At world 1 it is skipped unless ``force`` (the
        1-rank RCCL test issues the collective, captured, on the one GPU a box has)."""
        up = dist.is_available() and dist.is_initialized()
        if up and (force or dist.get_world_size(group) > 1):
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)
            self.flat.div_(dist.get_world_size(group))
        return self.flat
