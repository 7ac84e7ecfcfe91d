"""HRegNet training forward (train-mode BatchNorm) with its backward on the HIP library.

The reference trains ``HRegNet`` (models/HRegNet/models.py:77-148 with every
BatchNorm in .train(), train/train_reg_v0.py:241-296) through PyTorch autograd.
Here the same graph is built from ``torch.autograd.Function`` objects whose forward
and backward are C-ABI launches (csrc/train_ops.hip, csrc/train.hip, csrc/gemm.hip):
torch keeps the autograd tape, allocates memory and adds the gradients of tensors
used twice; every arithmetic op on the path runs in libhregnet_amd.so.

Layer structure follows the reference exactly, because train-mode BN needs the
batch statistics of every conv output before the next layer (the eval-mode fused
kernels of engine.py fold BN and cannot be used): conv -> BN(batch stats) -> ReLU
per layer (train.conv_bn_act), the reference's concatenations materialised as
row blocks, and each knn_gather / gather_operation a differentiable row gather whose
backward is a deterministic scatter (ascending destination order).

As in the reference, feature_extraction runs separately on src and dst (BN
statistics and running-stat updates per call, models.py:79-80) and so does the
CoarseReg neighbour branch (convs_2 on src, then dst: layers.py:334-343).
Index selections (FPS/WFPS, every kNN) are not differentiable (models/utils.py:33,
57; pytorch3d's knn_points indices) and run on the eval kernels; an ``IndexHook``
can record them or substitute given ones (parity tests pin the graph on the
reference's own selections).
"""
from __future__ import annotations

import torch

from . import _lib, engine, train
from ._lib import call

_f32 = torch.float32


def _stream():
    return _lib.stream_handle()


def _empty(*shape, dtype=_f32, device):
    return torch.empty(shape, dtype=dtype, device=device)


def _rows_ld(t):
    """(t, its row stride) for a [rows][C] gradient that may be a column view of a wider
    row block (_CatRows' backward); anything else is made contiguous"""
    if t.dim() == 2 and t.stride(1) == 1 and t.stride(0) >= t.shape[1]:
        return t, t.stride(0)
    t = t.contiguous()
    return t, t.shape[-1]


# ------------------------------------------------------------------ index maps

class IndexMap:
    """A gather index (global rows of a [n][C] source) plus its inverse, built on
    first use by a backward and shared by every gather through the same index."""

    def __init__(self, idx: torch.Tensor, n: int):
        assert idx.dtype == torch.int32 and idx.is_contiguous()
        self.idx = idx
        self.M = idx.numel()
        self.n = int(n)
        self._ws = None

    def csr(self):
        if self._ws is None:
            nbytes = _lib.load().hreg_csr_ws_bytes(self.M, self.n)
            self._ws = torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=self.idx.device)
            call("hreg_csr_build", self.idx, self.M, self.n, self._ws, _stream())
        return self._ws


def offset_index(local: torch.Tensor, n: int) -> torch.Tensor:
    """[nb, m(, k)] per-cloud indices -> flat int32 global rows of the [nb*n] stack."""
    local = local.to(torch.int32).contiguous()
    nb = local.shape[0]
    m = local.numel() // max(nb, 1)
    out = torch.empty(local.numel(), dtype=torch.int32, device=local.device)
    call("hreg_index_offset", local, nb, m, n, out, _stream())
    return out


class IndexHook:
    """Records every index selection of a training forward (``record``) and/or
    replaces it (``inject``: name -> per-cloud indices [nb, m(, k)], as the reference's
    fps / knn_points calls return them)."""

    def __init__(self, inject: dict | None = None, prepared: dict | None = None):
        self.inject = dict(inject or {})
        # name -> (local [nb, m] or None, global rows int32): selections already on the
        # device (the trainer's prefetched level-1 grouping), used without a copy
        self.prepared = dict(prepared or {})
        self.record = {}

    def __call__(self, name, local_fn, n, device):
        if name in self.inject:
            loc = torch.as_tensor(self.inject[name]).to(device=device, dtype=torch.int32)
        else:
            loc = local_fn()
        self.record[name] = loc
        return loc

    def record_global(self, name, gidx, nb, n):
        """record global rows as per-cloud indices [nb, m, ...] (test bookkeeping)"""
        g = gidx.view(nb, -1).to(torch.int64)
        off = torch.arange(nb, device=g.device, dtype=torch.int64)[:, None] * n
        self.record[name] = (g - off).to(torch.int32)


def _select(hook, name, local_fn, n, device, nb=None):
    """-> (local [nb, m(, k)] int32, IndexMap over global rows)."""
    if hook is not None and name in hook.prepared:
        loc, gidx = hook.prepared[name]
        return loc, IndexMap(gidx, nb * n)
    loc = hook(name, local_fn, n, device) if hook is not None else local_fn()
    return loc, IndexMap(offset_index(loc, n), loc.shape[0] * n)


# ------------------------------------------------------------ autograd functions

class _GatherRows(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, imap: IndexMap):
        n, C = x.shape
        out = _empty(imap.M, C, device=x.device)
        call("hreg_gather_rows", x, C, imap.idx, imap.M, C, out, C, _stream())
        ctx.imap = imap
        ctx.C = C
        return out

    @staticmethod
    def backward(ctx, dout):
        imap = ctx.imap
        dout, ldd = _rows_ld(dout)
        dx = _empty(imap.n, ctx.C, device=dout.device)
        call("hreg_scatter_rows", dout, ldd, imap.csr(), imap.M, imap.n, ctx.C, dx, ctx.C, 0,
             _stream())
        return dx, None


def gather_rows(x, imap: IndexMap):
    """out[m] = x[idx[m]] (knn_gather / gather_operation), x [n][C]."""
    return _GatherRows.apply(x.contiguous(), imap)


class _GeomRows(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, kx, k):
        G = q.shape[0]
        out = _empty(G * k, 4, device=q.device)
        call("hreg_geom_rows", q, kx, G, k, out, 4, _stream())
        ctx.save_for_backward(out)
        ctx.k = k
        return out

    @staticmethod
    def backward(ctx, dgeom):
        (geom,) = ctx.saved_tensors
        k = ctx.k
        G = geom.shape[0] // k
        dgeom, lddg = _rows_ld(dgeom)
        dq = _empty(G, 3, device=geom.device) if ctx.needs_input_grad[0] else None
        dkx = _empty(G * k, 3, device=geom.device) if ctx.needs_input_grad[1] else None
        call("hreg_geom_rows_bwd", geom, 4, dgeom, lddg, None, G, k, dq, dkx, _stream())
        return dq, dkx, None


def geom_rows(q, kx, k):
    """[knn_xyz - q, |knn_xyz - q|] per neighbour row (layers.py:21-23)."""
    return _GeomRows.apply(q.contiguous(), kx.contiguous(), k)


class _CatRows(torch.autograd.Function):
    """torch.cat over channels of row blocks; an input with repeat k is one row per
    group of k output rows (the reference's unsqueeze(2).repeat(1,1,k,1))."""

    @staticmethod
    def forward(ctx, reps, *xs):
        R = None
        for x, r in zip(xs, reps):
            rows = x.shape[0] * r
            assert R is None or rows == R, "row counts of the concatenated blocks differ"
            R = rows
        Ct = sum(x.shape[1] for x in xs)
        out = _empty(R, Ct, device=xs[0].device)
        c0 = 0
        for x, r in zip(xs, reps):
            C = x.shape[1]
            call("hreg_copy_rows", x, C, r, R, C, out[:, c0:], Ct, 0, _stream())
            c0 += C
        ctx.reps = reps
        ctx.widths = [x.shape[1] for x in xs]
        ctx.R = R
        return out

    @staticmethod
    def backward(ctx, dout):
        dout = dout.contiguous()
        Ct = dout.shape[1]
        grads = []
        c0 = 0
        for i, (C, r) in enumerate(zip(ctx.widths, ctx.reps)):
            if not ctx.needs_input_grad[1 + i]:
                grads.append(None)
            elif r == 1:
                # the block's columns of dout as a strided view (no copy): the consumers'
                # backward kernels take the row stride (_rows_ld)
                grads.append(dout[:, c0:c0 + C])
            else:
                g = _empty(ctx.R // r, C, device=dout.device)
                call("hreg_group_sum", dout[:, c0:], Ct, ctx.R // r, r, C, g, C, 0, _stream())
                grads.append(g)
            c0 += C
        return (None, *grads)


def cat_rows(*blocks):
    """blocks: tensors [R][C] or (tensor [G][C], k) repeated over k consecutive rows."""
    xs, reps = [], []
    for b in blocks:
        if isinstance(b, tuple):
            xs.append(b[0].contiguous())
            reps.append(int(b[1]))
        else:
            xs.append(b.contiguous())
            reps.append(1)
    return _CatRows.apply(tuple(reps), *xs)


class _Attention(torch.autograd.Function):
    """a = softmax_k(max_C logits); kp = sum_k a * knn_xyz; vmap = vals * a;
    vsum = sum_k vmap (layers.py:151-159 / 340-343 / 384-388 / 447-450)."""

    @staticmethod
    def forward(ctx, logits, vals, kx, k, same, want_map, want_sum):
        R, C = logits.shape
        G = R // k
        dev = logits.device
        v = logits if same else vals
        Cv = v.shape[1] if v is not None else 0
        a = _empty(R, device=dev)
        amax = _empty(R, dtype=torch.int32, device=dev)
        kp = _empty(G, 3, device=dev) if kx is not None else None
        vmap = _empty(R, Cv, device=dev) if (want_map and v is not None) else None
        vsum = _empty(G, Cv, device=dev) if (want_sum and v is not None) else None
        call("hreg_attention_fwd", logits, C, C, v, Cv, Cv, kx, G, k, a, amax, kp, vmap, Cv,
             vsum, Cv, _stream())
        ctx.save_for_backward(logits, vals, kx, a, amax)
        ctx.k, ctx.same = k, same
        ctx.set_materialize_grads(False)
        return kp, vmap, vsum

    @staticmethod
    def backward(ctx, dkp, dvmap, dvsum):
        logits, vals, kx, a, amax = ctx.saved_tensors
        k, same = ctx.k, ctx.same
        R, C = logits.shape
        G = R // k
        dev = logits.device
        v = logits if same else vals
        Cv = v.shape[1] if v is not None else 0
        dkp = dkp.contiguous() if dkp is not None else None
        dvmap, lddm = _rows_ld(dvmap) if dvmap is not None else (None, Cv)
        dvsum = dvsum.contiguous() if dvsum is not None else None
        dlogits = _empty(R, C, device=dev)
        dvals = _empty(R, Cv, device=dev) if (not same and vals is not None and
                                              ctx.needs_input_grad[1]) else None
        dkx = _empty(R, 3, device=dev) if (kx is not None and dkp is not None and
                                           ctx.needs_input_grad[2]) else None
        if dvals is not None and dvmap is None and dvsum is None:
            dvals.zero_()
        call("hreg_attention_bwd", logits, C, C, v, Cv, Cv, kx, G, k, a, amax, dkp, dvmap, lddm,
             dvsum, Cv, 1 if same else 0, dlogits, C, dvals, Cv, dkx, _stream())
        return dlogits, dvals, dkx, None, None, None, None


def attention(logits, k, vals=None, kx=None, want_map=False, want_sum=False):
    """-> (kp [G][3] | None, vmap [R][Cv] | None, vsum [G][Cv] | None); vals=None means
    the attention weights multiply the logits themselves."""
    same = vals is None
    return _Attention.apply(logits.contiguous(), None if same else vals.contiguous(),
                            None if kx is None else kx.contiguous(), k, same, want_map,
                            want_sum)


class _GroupMax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k):
        R, C = x.shape
        G = R // k
        out = _empty(G, C, device=x.device)
        arg = _empty(G, C, dtype=torch.int32, device=x.device)
        call("hreg_group_max_arg", x, C, G, k, C, out, C, arg, _stream())
        ctx.save_for_backward(arg)
        ctx.k, ctx.R = k, R
        return out

    @staticmethod
    def backward(ctx, dout):
        (arg,) = ctx.saved_tensors
        dout = dout.contiguous()
        G, C = dout.shape
        dx = _empty(ctx.R, C, device=dout.device)
        call("hreg_group_max_bwd", dout, C, arg, G, ctx.k, C, dx, C, 0, _stream())
        return dx, None


def group_max(x, k):
    """torch.max over each group of k rows (layers.py:202, 208)."""
    return _GroupMax.apply(x.contiguous(), k)


class _DescTail(torch.autograd.Function):
    """x2 = max over each group of k rows of x1 (layers.py:202), then
    cat([x2 repeated over the group's k rows, x1, att_map]) (layers.py:204-206) as one
    function: x1 feeds both, and its gradient is the concatenation's x1 columns with the
    group-max gradient added at each group's argmax rows (group_max_bwd accumulating into
    the copy) -- no dense zero-filled max gradient and no separate addition (autograd's
    sum of the two uses: the same fp32 additions)."""

    @staticmethod
    def forward(ctx, x1, att_map, k):
        R, C1 = x1.shape
        Ca = att_map.shape[1]
        G = R // k
        dev = x1.device
        x2 = _empty(G, C1, device=dev)
        arg = _empty(G, C1, dtype=torch.int32, device=dev)
        call("hreg_group_max_arg", x1, C1, G, k, C1, x2, C1, arg, _stream())
        Ct = 2 * C1 + Ca
        y = _empty(R, Ct, device=dev)
        call("hreg_copy_rows", x2, C1, k, R, C1, y, Ct, 0, _stream())
        call("hreg_copy_rows", x1, C1, 1, R, C1, y[:, C1:], Ct, 0, _stream())
        call("hreg_copy_rows", att_map, Ca, 1, R, Ca, y[:, 2 * C1:], Ct, 0, _stream())
        ctx.save_for_backward(arg)
        ctx.dims = (R, C1, Ca, k)
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        R, C1, Ca, k = ctx.dims
        G = R // k
        dy = dy.contiguous()
        Ct = dy.shape[1]
        dev = dy.device
        dx1 = dx2 = None
        if ctx.needs_input_grad[0]:
            dx2 = _empty(G, C1, device=dev)
            call("hreg_group_sum", dy, Ct, G, k, C1, dx2, C1, 0, _stream())
            dx1 = _empty(R, C1, device=dev)
            call("hreg_copy_rows", dy[:, C1:], Ct, 1, R, C1, dx1, C1, 0, _stream())
            call("hreg_group_max_bwd", dx2, C1, arg, G, k, C1, dx1, C1, 1, _stream())
        datt = dy[:, 2 * C1:] if ctx.needs_input_grad[1] else None
        return dx1, datt, None


def desc_tail(x1, att_map, k):
    return _DescTail.apply(x1.contiguous(), att_map.contiguous(), k)


class _HeadOut(torch.autograd.Function):
    """mlp3 (Conv1d C->1) + softplus + 0.001 (layers.py:161-163) or sigmoid
    (layers.py:393-394, 451-452); optionally the next level's WFPS weights
    (1/(sigma+1e-5))/mean (models.py:30-32) as a non-differentiable output."""

    @staticmethod
    def forward(ctx, x, w3, b3, mode, nclouds, rows, want_weights, params=(None, None)):
        G, C = x.shape
        out = _empty(G, device=x.device)
        wout = _empty(G, device=x.device) if want_weights else None
        call("hreg_head_out", x, C, C, nclouds, rows, w3, b3, mode, out, wout, _stream())
        ctx.save_for_backward(x, w3, b3)
        ctx.mode = mode
        # the conv's parameters (w3 is a view of the weight): their gradients are added
        # straight into the attached bucket when it is there (train._grad_slot)
        ctx.params, ctx.side = params, train._SIDE
        if wout is not None:
            ctx.mark_non_differentiable(wout)
        return out, wout

    @staticmethod
    def backward(ctx, dy, _dw):
        x, w3, b3 = ctx.saved_tensors
        G, C = x.shape
        dev = x.device
        dy = dy.contiguous()
        dz = _empty(G, 1, device=dev)
        dx = _empty(G, C, device=dev)
        call("hreg_head_out_bwd", x, C, C, w3, b3, dy, ctx.mode, G, dz, dx, C, _stream())
        dw = db = None
        if ctx.needs_input_grad[1]:
            gw = train._grad_slot(ctx.params[0], ctx.side)
            if gw is not None:
                train.gemm_tn(dz, x, into=gw.view(1, C))
            else:
                dw = train.gemm_tn(dz, x).view(-1)
        if ctx.needs_input_grad[2]:
            gb = train._grad_slot(ctx.params[1], ctx.side)
            if gb is not None:
                train.col_sum(dz, into=gb)
            else:
                db = train.col_sum(dz)
        return dx, dw, db, None, None, None, None, None


def head_out(x, conv, mode, nclouds=1, rows=None, want_weights=False):
    C = x.shape[1]
    w3 = conv.weight.view(C)
    return _HeadOut.apply(x.contiguous(), w3, conv.bias, mode, nclouds,
                          rows if rows is not None else x.shape[0], want_weights,
                          (conv.weight, conv.bias))


class _SimFeats(torch.autograd.Function):
    """[src_dst_cos, dst_src_cos] gathered at the descriptor kNN (layers.py:290-313)."""

    @staticmethod
    def forward(ctx, a, b, kidx, nb, N1, N2):
        C = a.shape[1]
        dev = a.device
        k = kidx.shape[-1]
        na = _empty(nb * N1, device=dev)
        nbv = _empty(nb * N2, device=dev)
        call("hreg_row_norms", a, nb * N1, C, C, na, _stream())
        call("hreg_row_norms", b, nb * N2, C, C, nbv, _stream())
        S = _empty(nb, N1, N2, device=dev)
        engine.cosine_gemm(a, b, na, nbv, nb, N1, N2, C, S)
        rmax = _empty(nb * N1, device=dev)
        rarg = _empty(nb * N1, dtype=torch.int32, device=dev)
        cmax = _empty(nb * N2, device=dev)
        carg = _empty(nb * N2, dtype=torch.int32, device=dev)
        call("hreg_sim_stats", S, nb, N1, N2, rmax, rarg, cmax, carg, _stream())
        out = _empty(nb * N1 * k, 2, device=dev)
        call("hreg_sim_feats", S, nb, N1, N2, kidx, k, rmax, cmax, out, 2, _stream())
        ctx.save_for_backward(a, b, kidx, na, nbv, S, rmax, rarg, cmax, carg)
        ctx.dims = (nb, N1, N2, C, k)
        return out

    @staticmethod
    def backward(ctx, dout):
        a, b, kidx, na, nbv, S, rmax, rarg, cmax, carg = ctx.saved_tensors
        nb, N1, N2, C, k = ctx.dims
        dev = a.device
        ws = torch.empty(_lib.load().hreg_sim_feats_bwd_ws_bytes(nb, N1, N2), dtype=torch.uint8,
                         device=dev)
        da = _empty(nb * N1, C, device=dev)
        db = _empty(nb * N2, C, device=dev)
        dout, ldd = _rows_ld(dout)
        call("hreg_sim_feats_bwd", S, a, b, na, nbv, nb, N1, N2, C, kidx, k, rmax, rarg, cmax,
             carg, dout, ldd, ws, da, db, _stream())
        return da, db, None, None, None, None


def sim_feats(a, b, kidx, nb, N1, N2):
    return _SimFeats.apply(a.contiguous(), b.contiguous(), kidx.contiguous(), nb, N1, N2)


class _WeightedSVD(torch.autograd.Function):
    @staticmethod
    def forward(ctx, src, corres, w):
        B, n, _ = src.shape
        _, _, R, t = engine.weighted_svd(src, corres, w)
        ctx.save_for_backward(src, corres, w)
        return R, t

    @staticmethod
    def backward(ctx, dR, dt):
        src, corres, w = ctx.saved_tensors
        B, n, _ = src.shape
        dev = src.device
        dR = torch.zeros(B, 3, 3, device=dev) if dR is None else dR.contiguous()
        dt = torch.zeros(B, 3, device=dev) if dt is None else dt.contiguous()
        ds = torch.empty_like(src)
        dc = torch.empty_like(corres)
        dw = torch.empty_like(w)
        call("hreg_weighted_svd_bwd", src, corres, w, B, n, dR, dt, ds, dc, dw, _stream())
        return ds, dc, dw


def weighted_svd(src, corres, w):
    """WeightedSVDHead (layers.py:469-504): (R [B,3,3], t [B,3])."""
    return _WeightedSVD.apply(src.contiguous(), corres.contiguous(), w.contiguous())


class _Transform(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xyz, R, t):
        B, n, _ = xyz.shape
        out = torch.empty_like(xyz)
        call("hreg_transform_points", xyz, R, t, B, n, out, _stream())
        ctx.save_for_backward(xyz, R)
        return out

    @staticmethod
    def backward(ctx, dy):
        xyz, R = ctx.saved_tensors
        B, n, _ = xyz.shape
        dev = xyz.device
        dx = torch.empty_like(xyz) if ctx.needs_input_grad[0] else None
        dR = _empty(B, 3, 3, device=dev)
        dt = _empty(B, 3, device=dev)
        call("hreg_transform_points_bwd", xyz, R, B, n, dy.contiguous(), dx, dR, dt, _stream())
        return dx, dR, dt


def transform(xyz, R, t):
    """R xyz^T + t (models.py:91-92, 113-114)."""
    return _Transform.apply(xyz.contiguous(), R.contiguous(), t.contiguous())


class _Compose(torch.autograd.Function):
    @staticmethod
    def forward(ctx, Ra, ta, Rb, tb):
        B = Ra.shape[0]
        Ro = torch.empty_like(Ra)
        to = torch.empty_like(ta)
        call("hreg_compose_se3", B, Ra, ta, Rb, tb, Ro, to, _stream())
        ctx.save_for_backward(Ra, Rb, tb)
        return Ro, to

    @staticmethod
    def backward(ctx, dRo, dto):
        Ra, Rb, tb = ctx.saved_tensors
        B = Ra.shape[0]
        dev = Ra.device
        dRo = torch.zeros(B, 3, 3, device=dev) if dRo is None else dRo.contiguous()
        dto = torch.zeros(B, 3, device=dev) if dto is None else dto.contiguous()
        dRa, dRb = torch.empty_like(Ra), torch.empty_like(Rb)
        dta, dtb = _empty(B, 3, device=dev), torch.empty_like(tb)
        call("hreg_compose_se3_bwd", B, Ra, Rb, tb, dRo, dto, dRa, dta, dRb, dtb, _stream())
        return dRa, dta, dRb, dtb


def compose(Ra, ta, Rb, tb):
    """T = T_a @ T_b (models.py:100-110): (Ra Rb, Ra tb + ta)."""
    return _Compose.apply(Ra.contiguous(), ta.contiguous(), Rb.contiguous(), tb.contiguous())


class _TransformationLoss(torch.autograd.Function):
    """transformation_loss(...)[0] = alpha * mean |R^T R_gt - I|_F + mean |t - t_gt|
    (losses/losses.py:117-160); also returns (loss_R, loss_t) without gradient."""

    @staticmethod
    def forward(ctx, R, t, gR, gt, alpha):
        B = R.shape[0]
        dev = R.device
        scal = _empty(3, device=dev)
        R_err = _empty(3, device=dev)
        T_err = _empty(3, device=dev)
        call("hreg_transformation_loss", R, t, gR, gt, B, float(alpha), scal, R_err, T_err, None,
             None, _stream())
        ctx.save_for_backward(R, t, gR, gt)
        ctx.alpha = float(alpha)
        parts = scal[1:].clone()
        ctx.mark_non_differentiable(parts)
        return scal[0].clone(), parts

    @staticmethod
    def backward(ctx, dloss, _dparts):
        R, t, gR, gt = ctx.saved_tensors
        B = R.shape[0]
        dR = torch.empty_like(R)
        dt = torch.empty_like(t)
        call("hreg_transformation_loss_bwd", R, t, gR, gt, B, ctx.alpha, 1.0,
             dloss.contiguous().view(1), dR, dt, _stream())
        return dR, dt, None, None, None


def transformation_loss(R, t, gR, gt, alpha=1.0):
    """-> (loss, [loss_R, loss_t]) with loss differentiable in R and t."""
    return _TransformationLoss.apply(R.contiguous(), t.contiguous(), gR.contiguous(),
                                     gt.contiguous(), alpha)


# ------------------------------------------------------------------ modules

_BN_COUNTERS: list = []  # num_batches_tracked of every BN call of the current forward


def _flush_bn_counters():
    """num_batches_tracked += 1 per BN call, as one multi-tensor launch per forward (a
    module called twice -- src and dst -- appears once, with its count)."""
    if _BN_COUNTERS:
        uniq = {}
        for t in _BN_COUNTERS:
            uniq.setdefault(id(t), [t, 0])[1] += 1
        torch._foreach_add_([t for t, _ in uniq.values()], [c for _, c in uniq.values()])
        _BN_COUNTERS.clear()


# the descriptor's mlp1 without its input concatenation (train.tail_conv_bn_act, r6; bitwise the
# concatenation path, which stays as the test checker and for shapes its kernels do not take)
TAIL_FUSED = True


def conv_bn(x, conv, bn, relu=True):
    """Conv(1x1) + train-mode BatchNorm (+ ReLU) over rows (num_batches_tracked += 1)."""
    W = conv.weight.view(conv.out_channels, -1)
    y = train.conv_bn_act(x, W, conv.bias, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                          relu, momentum=bn.momentum, eps=bn.eps, wparam=conv.weight)
    if bn.num_batches_tracked is not None:
        _BN_COUNTERS.append(bn.num_batches_tracked)
    return y


def _layer(conv, bn):
    """a (Conv, BN) pair as train.conv_bn_chain's layer tuple"""
    return (conv.weight.view(conv.out_channels, -1), conv.bias, bn.weight, bn.bias, bn.running_mean,
            bn.running_var, bn.momentum, bn.eps, conv.weight)


def _count_bn(*bns):
    """num_batches_tracked += 1 for each BN called (flushed once per forward)"""
    for bn in bns:
        if bn.num_batches_tracked is not None:
            _BN_COUNTERS.append(bn.num_batches_tracked)


def _pairs(seq):
    """nn.Sequential of [Conv, BN, ReLU] * n -> [(conv, bn)]"""
    mods = list(seq)
    return [(mods[i], mods[i + 1]) for i in range(0, len(mods), 3)]


def conv_bn_seq(x, pairs):
    """[(conv, bn)] each Conv(1x1) + train-mode BN + ReLU in order: one fused chain
    (train.conv_bn_chain: the inner activations never written, the same bits) when its kernels
    take the shapes, else layer by layer."""
    widths = [x.shape[1]] + [conv.out_channels for conv, _ in pairs]
    if len(pairs) >= 2 and train.chain_fusable(x.shape[0], widths):
        y = train.conv_bn_chain(x, [_layer(c, b) for c, b in pairs])
        _count_bn(*(b for _, b in pairs))
        return y
    for conv, bn in pairs:
        x = conv_bn(x, conv, bn, relu=True)
    return x


def seq_convs(x, seq):
    """nn.Sequential of [Conv, BN, ReLU] * n."""
    return conv_bn_seq(x, _pairs(seq))


def _mlp_head(x, head_mods, mode, nclouds, rows, want_weights=False):
    m1, m2, m3 = head_mods
    s = conv_bn_seq(x, [(m1[0], m1[1]), (m2[0], m2[1])])
    return head_out(s, m3[0], mode, nclouds, rows, want_weights)


def keypoint_level(det, desc, lvl, xyz, feats, weights, hook=None, part="src", use_fps=True):
    """KeypointDetector.forward + DescExtractor.forward (layers.py:134-209), train mode.

    xyz [nb,n,3] (requires grad above level 1), feats [nb*n][Cf] or None, weights [nb*n]
    (WFPS, no gradient) or None.  -> keypoints [nb,M,3], sigmas [nb*M], att_feat
    [nb*M][C], desc [nb*M][Cd], next weights [nb*M] (no gradient)."""
    M, k = engine.LEVELS[lvl][:2]
    nb, n, _ = xyz.shape
    dev = xyz.device
    G = nb * M
    xyz_flat = xyz.reshape(nb * n, 3)
    with torch.no_grad():
        xd = xyz.detach().contiguous()
        wd = None if weights is None else weights.detach().view(nb, n).contiguous()
        grouped = []

        def fps_local():
            if not use_fps:  # layers.py:144-147: one host randperm draw for the batch
                return engine.random_sample_level(lvl, n, nb, dev)
            grouped.append(engine.grouping(xd, lvl, wd))  # FPS/WFPS + kNN grouping
            return grouped[0][0]

        fps_loc, fps_map = _select(hook, f"{part}_fps_{lvl + 1}", fps_local, n, dev, nb)
        knn_name = f"{part}_knn_{lvl + 1}"
        if hook is not None and knn_name in hook.prepared:
            _, kmap = _select(hook, knn_name, None, n, dev, nb)
        elif grouped and not (hook is not None and knn_name in hook.inject):
            kmap = IndexMap(grouped[0][2].contiguous(), nb * n)  # global rows
            if hook is not None:
                hook.record_global(knn_name, kmap.idx, nb, n)
        else:
            q_sel = _empty(nb, M, 3, device=dev)
            call("hreg_gather_rows", xd.view(nb * n, 3), 3, fps_map.idx, G, 3, q_sel, 3,
                 _stream())
            _, kmap = _select(hook, knn_name, lambda: engine.knn_idx32(q_sel, xd, k), n, dev)
    # differentiable recomputation of the grouped rows (layers.py:19-27, 139-149)
    q = gather_rows(xyz_flat, fps_map)                  # sampled_xyz [G][3]
    kx = gather_rows(xyz_flat, kmap)                    # knn_xyz [R][3]
    geom = geom_rows(q, kx, k)                          # [rela, dist]
    if feats is not None:
        grouped_rows = cat_rows(geom, gather_rows(feats, kmap))
    else:
        grouped_rows = geom
    # detector (layers.py:150-165)
    dpairs = _pairs(det.convs)
    if k <= 64 and train.chain_fusable(grouped_rows.shape[0],
                                       [grouped_rows.shape[1]] + [c.out_channels for c, _ in dpairs]):
        # the detector's convs and its attention with the last activation never written (the same bits)
        kp, att_map, att_feat = train.conv_bn_chain_attention(grouped_rows, [_layer(c, b) for c, b in dpairs],
                                                              k, kx)
        _count_bn(*(b for _, b in dpairs))
    else:
        emb = seq_convs(grouped_rows, det.convs)
        kp, att_map, att_feat = attention(emb, k, kx=kx, want_map=True, want_sum=True)
    sig, wnext = _mlp_head(att_feat, (det.mlp1, det.mlp2, det.mlp3), _lib.HREG_HEAD_SOFTPLUS,
                           nb, M, want_weights=True)
    # descriptor (layers.py:200-209)
    x1 = seq_convs(grouped_rows, desc.convs)
    conv, bn = desc.mlp1[0], desc.mlp1[1]
    conv2, bn2 = desc.mlp2[0], desc.mlp2[1]
    if TAIL_FUSED and train.tail_chain_fusable(x1.shape[0], k, x1.shape[1], att_map.shape[1],
                                               [conv.out_channels, conv2.out_channels]):
        # mlp1 without its input concatenation, mlp2 applying mlp1's BN + ReLU on load and the k-max
        # mlp2's (the same bits as the layerwise path)
        d = train.tail_conv_bn_chain(x1, att_map, k, _layer(conv, bn), [_layer(conv2, bn2)], group_max=True)
        _count_bn(bn, bn2)
        return kp.view(nb, M, 3), sig, att_feat, d, wnext, fps_loc
    if TAIL_FUSED and train.tail_fusable(x1.shape[0], k, x1.shape[1], att_map.shape[1], conv.out_channels):
        # mlp1 over cat([max_k x1 repeated, x1, att_map]) without materialising it (the same bits)
        y = train.tail_conv_bn_act(x1, att_map, k, conv.weight.view(conv.out_channels, -1), conv.bias,
                                   bn.weight, bn.bias, bn.running_mean, bn.running_var, momentum=bn.momentum,
                                   eps=bn.eps, wparam=conv.weight)
        if bn.num_batches_tracked is not None:
            _BN_COUNTERS.append(bn.num_batches_tracked)
    else:
        y = desc_tail(x1, att_map, k)  # cat([max_k x1 repeated, x1, att_map])
        y = conv_bn(y, conv, bn)
    y = conv_bn(y, desc.mlp2[0], desc.mlp2[1])
    d = group_max(y, k)
    return kp.view(nb, M, 3), sig, att_feat, d, wnext, fps_loc


def feature_extraction(fe, points, hook=None, part="src"):
    """HierFeatureExtraction.forward (models.py:26-58) in train mode."""
    dets = (fe.detector_1, fe.detector_2, fe.detector_3)
    descs = (fe.desc_extractor_1, fe.desc_extractor_2, fe.desc_extractor_3)
    out = {}
    xyz, feats, w = points, None, None
    for lvl in range(3):
        kp, sig, att, d, wnext, fps_loc = keypoint_level(dets[lvl], descs[lvl], lvl, xyz, feats,
                                                         w, hook, part, fe.use_fps)
        M = engine.LEVELS[lvl][0]
        nb = points.shape[0]
        out[f"xyz_{lvl + 1}"] = kp
        out[f"sigmas_{lvl + 1}"] = sig.view(nb, M)
        out[f"desc_{lvl + 1}"] = d  # [nb*M][C] point-major
        out[f"fps_idx_{lvl + 1}"] = fps_loc
        xyz, feats = kp, att
        w = wnext if fe.use_weights else None
    return out


def feature_extraction_call(fe, points):
    """HierFeatureExtraction called by itself in train mode (train_feats.py's use): the
    forward above plus the BN num_batches_tracked bumps hregnet_train_forward makes once per
    forward (one per BN call)."""
    _BN_COUNTERS.clear()
    out = feature_extraction(fe, points)
    _flush_bn_counters()
    return out


def _knn_local(hook, name, p1, p2, k, dev):
    loc = hook(name, lambda: engine.knn_idx32(p1, p2, k), p2.shape[1], dev) if hook is not None \
        else engine.knn_idx32(p1, p2, k)
    return loc


def _nbr_desc(convs_2, xyz, desc, k, hook, name):
    """Neighbour-aware descriptor of one cloud set (layers.py:315-343)."""
    nb, N, _ = xyz.shape
    dev = xyz.device
    with torch.no_grad():
        xd = xyz.detach().contiguous()
        loc = _knn_local(hook, name, xd, xd, k, dev)
        imap = IndexMap(offset_index(loc, N), nb * N)
    xyz_flat = xyz.reshape(nb * N, 3)
    kfeat = gather_rows(desc, imap)                        # src_nbr_knn_feats
    kx = gather_rows(xyz_flat, imap)
    rows = cat_rows(kfeat, geom_rows(xyz_flat, kx, k))     # [knn_feats, rela, dist]
    h = seq_convs(rows, convs_2)
    _, _, nbr = attention(h, k, vals=kfeat, want_sum=True)
    return nbr


def coarse_reg(m, s_xyz, s_desc, d_xyz, d_desc, s_w, d_w, hook=None, keep=None):
    """CoarseReg.forward (layers.py:273-396), train mode.  xyz [B,N,3], desc [B*N][C]
    point-major, w [B*N] (the sigmas, models.py:84-85).  keep (a list; the two-stream step):
    the src neighbour branch on the side stream (gradient side 0), the dst one on the current
    stream (side 1, BN running updates queued into keep and applied after the src ones on the
    side stream; the caller joins it)."""
    if not (getattr(m, "use_sim", True) and getattr(m, "use_neighbor", True)):
        raise NotImplementedError("the training step builds CoarseReg(use_sim=True, use_neighbor=True) "
                                  "only (as HRegNet, models.py:71); the variants run in eval mode")
    k = m.k
    B, N1, _ = s_xyz.shape
    N2 = d_xyz.shape[1]
    C = s_desc.shape[1]
    dev = s_xyz.device
    with torch.no_grad():
        kidx = _knn_local(hook, "coarse_desc_knn", s_desc.detach().view(B, N1, C),
                          d_desc.detach().view(B, N2, C), k, dev)
        kmap = IndexMap(offset_index(kidx, N2), B * N2)
    s_flat = s_xyz.reshape(B * N1, 3)
    kx = gather_rows(d_xyz.reshape(B * N2, 3), kmap)                # src_knn_xyz
    geom = geom_rows(s_flat, kx, k)                                 # rela, dist
    kdesc = gather_rows(d_desc, kmap)                               # src_knn_desc
    kw = gather_rows(d_w.reshape(B * N2, 1), kmap)                  # src_knn_weights
    sims_a = sim_feats(s_desc, d_desc, kidx, B, N1, N2)             # original similarity
    if keep is not None:
        main = torch.cuda.current_stream()
        side = side_stream(s_xyz.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            nbr_s = _nbr_desc(m.convs_2, s_xyz, s_desc, k, hook, "coarse_nbr_src")
        with train.side(1, defer_running=True) as queued:
            nbr_d = _nbr_desc(m.convs_2, d_xyz, d_desc, k, hook, "coarse_nbr_dst")
        main.wait_stream(side)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            train.apply_running(queued)
        record_on((nbr_s,), main)                  # made on the side stream, read here
        for mean, var, _, _, _ in queued:
            record_on((mean, var), side)           # made here, read on the side stream
        keep.append(queued)
    else:
        nbr_s = _nbr_desc(m.convs_2, s_xyz, s_desc, k, hook, "coarse_nbr_src")
        nbr_d = _nbr_desc(m.convs_2, d_xyz, d_desc, k, hook, "coarse_nbr_dst")
    sims_b = sim_feats(nbr_s, nbr_d, kidx, B, N1, N2)               # neighbour-aware
    feats = cat_rows(geom, (s_flat, k), kx, (s_desc, k), kdesc, (s_w.reshape(B * N1, 1), k), kw,
                     sims_a, sims_b)
    f = seq_convs(feats, m.convs_1)
    corres, _, att = attention(f, k, kx=kx, want_sum=True)
    w, _ = _mlp_head(att, (m.mlp1, m.mlp2, m.mlp3), _lib.HREG_HEAD_SIGMOID, 1, B * N1)
    return corres.view(B, N1, 3), w.view(B, N1)


def fine_reg(m, s_xyz, s_feat, d_xyz, d_feat, s_w, d_w, hook=None, name="fine", return_att=False):
    """FineReg.forward (layers.py:433-454), train mode (return_att: also the attentive
    features [B*N1][2C] that FineReg2 feeds to mlpx, model_v2/layers.py:484-490)."""
    k = m.k
    B, N1, _ = s_xyz.shape
    N2 = d_xyz.shape[1]
    dev = s_xyz.device
    with torch.no_grad():
        kidx = _knn_local(hook, name + "_knn", s_xyz.detach().contiguous(),
                          d_xyz.detach().contiguous(), k, dev)
        kmap = IndexMap(offset_index(kidx, N2), B * N2)
    s_flat = s_xyz.reshape(B * N1, 3)
    kx = gather_rows(d_xyz.reshape(B * N2, 3), kmap)
    geom = geom_rows(s_flat, kx, k)
    kf = gather_rows(d_feat, kmap)
    kw = gather_rows(d_w.reshape(B * N2, 1), kmap)
    feats = cat_rows(geom, (s_flat, k), kx, (s_feat, k), kf, (s_w.reshape(B * N1, 1), k), kw)
    f = seq_convs(feats, m.convs_1)
    corres, _, att = attention(f, k, kx=kx, want_sum=True)
    w, _ = _mlp_head(att, (m.mlp1, m.mlp2, m.mlp3), _lib.HREG_HEAD_SIGMOID, 1, B * N1)
    if return_att:
        return corres.view(B, N1, 3), w.view(B, N1), att
    return corres.view(B, N1, 3), w.view(B, N1)


def batch_shuffle(x, perm):
    """x[perm] along the batch dimension (FineReg2's prime copies, model_v2/layers.py:492,
    497) as a row gather over [B][rest] with the deterministic scatter backward."""
    B = x.shape[0]
    rows = x.reshape(B, -1)
    imap = IndexMap(perm.to(device=x.device, dtype=torch.int32).contiguous(), B)
    return gather_rows(rows, imap).view_as(x)


_SIDE_STREAMS: dict = {}


def side_stream(device) -> "torch.cuda.Stream":
    """the stream the src feature extraction (and its backward) runs on in the two-stream step"""
    key = str(device)
    if key not in _SIDE_STREAMS:
        _SIDE_STREAMS[key] = torch.cuda.Stream(device=device)
    return _SIDE_STREAMS[key]


def join_side_stream(device) -> None:
    """the current stream waits for everything enqueued on the side stream (after the backward
    of a two-stream step: the src side's direct gradient additions ran there)"""
    key = str(device)
    if key in _SIDE_STREAMS:
        torch.cuda.current_stream().wait_stream(_SIDE_STREAMS[key])


def _two_stream_features(fe, src, dst, hook):
    """src feature extraction on the side stream (gradient side 0, its BN running statistics
    updated in the GEMM epilogues as it runs), dst on the current stream (side 1, running
    updates queued), joined; the dst updates then run on the side stream after the src ones
    -- the reference's order of the two calls of each module -- beside the heads."""
    main = torch.cuda.current_stream()
    s = side_stream(src.device)
    s.wait_stream(main)
    with torch.cuda.stream(s):
        sf = feature_extraction(fe, src, hook, "src")
    with train.side(1, defer_running=True) as queued:
        df = feature_extraction(fe, dst, hook, "dst")
    main.wait_stream(s)
    s.wait_stream(main)
    with torch.cuda.stream(s):
        train.apply_running(queued)
    # tensors crossing streams are recorded on the stream that reads them, so the allocator
    # cannot hand their blocks to another allocation before that stream is done with them:
    # the src features (made on the side stream, read on the current one) and the queued
    # statistics (made on the current stream, read on the side stream; a block freed early
    # here was a race a captured graph replayed: r3, running_var off by ~20 %).  They also
    # stay referenced until the caller's join.
    record_on(sf.values(), main)
    for mean, var, _, _, _ in queued:
        record_on((mean, var), s)
    return sf, df, queued


def record_on(tensors, stream) -> None:
    """t.record_stream(stream) for every tensor (a consumer on another stream than the
    producer's: the caching allocator then keeps the block until that stream's work is done)"""
    for t in tensors:
        if isinstance(t, torch.Tensor) and t.is_cuda:
            t.record_stream(stream)


def hregnet_train_forward(net, src, dst, hook=None, v2=False, concurrent=False):
    """HRegNet.forward (models/HRegNet/models.py:77-148) in train mode -> the reference's
    result dict; differentiable in every parameter that requires grad.  v2: Model_V2's
    forward (model_v2/models.py:77-183): fine_corres_2 is FineReg2, whose attentive
    features also pass mlpx (Conv1d + train-mode BN + ReLU) and whose prime copies are
    batch shuffles by two host torch.randperm(B) draws, features first
    (model_v2/layers.py:484-497); returns Model_V2's dict.  concurrent: the src and dst
    feature extractions on two streams (needs a GradBucket(sides=2) attached; the caller
    joins the side stream after the backward, join_side_stream) -- the same arithmetic and
    the same results as the serial order."""
    fe = net.feature_extraction
    src = src.float().contiguous()
    dst = dst.float().contiguous()
    B = src.shape[0]
    _BN_COUNTERS.clear()
    keep = None
    if concurrent:
        sf, df, queued = _two_stream_features(fe, src, dst, hook)
        keep = [queued]
    else:
        sf = feature_extraction(fe, src, hook, "src")
        df = feature_extraction(fe, dst, hook, "dst")
    c3, w3 = coarse_reg(net.coarse_corres, sf["xyz_3"], sf["desc_3"], df["xyz_3"], df["desc_3"],
                        sf["sigmas_3"], df["sigmas_3"], hook, keep)
    R3, t3 = weighted_svd(sf["xyz_3"], c3, w3)
    x2t = transform(sf["xyz_2"], R3, t3)
    if v2:
        m2 = net.fine_corres_2
        c2, w2, att2 = fine_reg(m2, x2t, sf["desc_2"], df["xyz_2"], df["desc_2"],
                                sf["sigmas_2"], df["sigmas_2"], hook, "fine2", return_att=True)
        N2 = c2.shape[1]
        f2 = conv_bn(att2, m2.mlpx[0], m2.mlpx[1], relu=True)       # [B*N2][C]
        feats2 = f2.view(B, N2, -1).transpose(1, 2)                   # [B, C, N2]
        pf, pw = torch.randperm(B), torch.randperm(B)                 # features first
        feats2_prime = batch_shuffle(f2.view(B, N2, -1), pf).transpose(1, 2)
        w2_prime = batch_shuffle(w2, pw)
    else:
        c2, w2 = fine_reg(net.fine_corres_2, x2t, sf["desc_2"], df["xyz_2"], df["desc_2"],
                          sf["sigmas_2"], df["sigmas_2"], hook, "fine2")
    R2_, t2_ = weighted_svd(x2t, c2, w2)
    R2, t2 = compose(R2_, t2_, R3, t3)
    x1t = transform(sf["xyz_1"], R2, t2)
    c1, w1 = fine_reg(net.fine_corres_1, x1t, sf["desc_1"], df["xyz_1"], df["desc_1"],
                      sf["sigmas_1"], df["sigmas_1"], hook, "fine1")
    R1_, t1_ = weighted_svd(x1t, c1, w1)
    R1, t1 = compose(R1_, t1_, R2, t2)
    _flush_bn_counters()
    if concurrent:
        join_side_stream(src.device)  # (the dst running-statistics updates)
        del keep

    def feats(f):
        d = {}
        for i, m in enumerate((1024, 512, 256)):
            d[f"xyz_{i + 1}"] = f[f"xyz_{i + 1}"]
            d[f"sigmas_{i + 1}"] = f[f"sigmas_{i + 1}"]
            d[f"desc_{i + 1}"] = f[f"desc_{i + 1}"].view(B, m, -1).transpose(1, 2)
        return d

    if v2:  # model_v2/models.py:143-181
        sfd, dfd = feats(sf), feats(df)
        return {
            "src_xyz_corres_3": c3, "src_xyz_corres_2": c2, "src_xyz_corres_1": c1,
            "rotation": [R3, R2, R1], "translation": [t3, t2, t1],
            "src_feats_desc_2": sfd["desc_2"], "src_feats_sigmas_2": sfd["sigmas_2"],
            "src_xyz_2_trans": x2t, "dst_xyz_2": dfd["xyz_2"],
            "src_dst_feats_2": feats2, "src_dst_feats_2_prime": feats2_prime,
            "src_dst_weights_2": w2, "src_dst_weights_2_prime": w2_prime,
            "src_feats": sfd, "dst_feats": dfd,
        }
    return {
        "src_xyz_corres_3": c3, "src_xyz_corres_2": c2, "src_xyz_corres_1": c1,
        "src_dst_weights_3": w3, "src_dst_weights_2": w2, "src_dst_weights_1": w1,
        "rotation": [R3, R2, R1], "translation": [t3, t2, t1],
        "src_feats": feats(sf), "dst_feats": feats(df),
    }


def registration_loss(ret, gt_R, gt_t, alpha=1.0):
    """train_reg_v0.py:280-294: l_trans = mean over the 3 levels of transformation_loss;
    -> (loss, l_R, l_t) with loss differentiable."""
    losses, lr, lt = [], [], []
    for R, t in zip(ret["rotation"], ret["translation"]):
        l, parts = transformation_loss(R, t, gt_R, gt_t, alpha)
        losses.append(l)
        lr.append(parts[0])
        lt.append(parts[1])
    return torch.stack(losses).sum() / 3.0, torch.stack(lr).sum() / 3.0, torch.stack(lt).sum() / 3.0
