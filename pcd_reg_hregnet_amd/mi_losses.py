"""Model_V2 training losses on the HIP library.

* ``ChamferDistanceLoss(scale, reduction)`` -- losses/chamfer_loss.py:10-36.  The
  reference wraps the third-party ``chamfer_distance`` CUDA extension (not vendored,
  not installed); its published semantics -- the squared distance from every point to
  its nearest neighbour in the other cloud, both directions -- run in
  ``hreg_chamfer`` (csrc/mi_loss.hip), then sqrt, per-cloud means, (a + b) / 2 and
  the batch reduction in one fixed-order block.  Forward only: the Model_V2 trainer
  uses it as a Python float (``c_loss.item()``, train/train_reg_v6.py:330-340), so no
  gradient flows through it.
* ``DeepMILoss(global_in_channels, local_in_channels)`` -- losses/mi_loss_v2.py:42-79,
  same submodules, parameter names and call convention (state dicts interchange with
  the reference's ``mi_loss_state_dict``).  The discriminators' 1x1 convs are fp32
  MFMA GEMMs (``hreg_gemm``; backward ``hreg_gemm_tn`` / ``hreg_gemm`` with W^T), the
  single-output layers ``hreg_rowdot``, the JS estimator ``hreg_js_loss``; joint and
  marginal pairs go through each discriminator in one batched pass.  Differentiable
  in its inputs and parameters (autograd Functions over the C ABI).

No CPU fallback: every op raises without the HIP library and a GPU.
"""
from __future__ import annotations

import math

import torch

from . import _lib, engine, train
from ._lib import call


def _stream():
    return _lib.stream_handle()


def _rows(x: torch.Tensor) -> torch.Tensor:
    """[B, C, N] (the reference's Conv1d layout) -> point rows [B*N, C]; [B, C] stays."""
    if not x.is_cuda:
        raise RuntimeError("pcd_reg_hregnet_amd.mi_losses: tensors must be on the GPU "
                           "(there is no CPU fallback)")
    if x.dim() == 3:
        return x.permute(0, 2, 1).reshape(-1, x.shape[1]).contiguous().float()
    return x.contiguous().float()


class _LinearAct(torch.autograd.Function):
    """y = [ReLU](x W^T + b) over rows (Conv1d k=1 / Linear)."""

    @staticmethod
    def forward(ctx, x, W, b, relu):
        N = W.shape[0]
        ones = train._const(1.0, N, x.device)
        shift = b if b is not None else train._const(0.0, N, x.device)
        y = engine.gemm([engine._seg(x, 0, x.shape[1])],
                        engine.Lin(W.contiguous(), ones, shift.contiguous(), relu=relu), x.shape[0])
        ctx.save_for_backward(x, W, y)
        ctx.relu = relu
        ctx.has_bias = b is not None
        return y

    @staticmethod
    def backward(ctx, dout):
        x, W, y = ctx.saved_tensors
        dy = dout.contiguous()
        if ctx.relu:
            g = torch.empty_like(dy)
            call("hreg_relu_bwd", dy, y, dy.numel(), g, _stream())
            dy = g
        dW = train.gemm_tn(dy, x) if ctx.needs_input_grad[1] else None
        db = train.col_sum(dy) if ctx.has_bias and ctx.needs_input_grad[2] else None
        dx = train._plain_gemm(dy, train.transpose(W), None) if ctx.needs_input_grad[0] else None
        return dx, dW, db, None


class _RowDot(torch.autograd.Function):
    """t = [ReLU](h w + b): the single-output conv3 / l0."""

    @staticmethod
    def forward(ctx, h, w, b, relu):
        R, C = h.shape
        t = torch.empty(R, device=h.device)
        call("hreg_rowdot", h, R, C, w, b, 1 if relu else 0, t, _stream())
        ctx.save_for_backward(h, w, t)
        ctx.relu = relu
        ctx.has_bias = b is not None
        return t

    @staticmethod
    def backward(ctx, g):
        h, w, t = ctx.saved_tensors
        R, C = h.shape
        g = g.contiguous()
        dh = torch.empty_like(h) if ctx.needs_input_grad[0] else None
        dw = torch.empty(C, device=h.device) if ctx.needs_input_grad[1] else None
        db = torch.empty(1, device=h.device) if ctx.has_bias and ctx.needs_input_grad[2] else None
        call("hreg_rowdot_bwd", g, t, 1 if ctx.relu else 0, h, R, C, w, dh, dw, db, _stream())
        return dh, dw, db, None


class _JS(torch.autograd.Function):
    """0.5 (Em - Ej) with Ej = -mean softplus(-t_joint), Em = mean softplus(t_marg)."""

    @staticmethod
    def forward(ctx, tj, tm):
        n = tj.shape[0]
        out = torch.empty(3, device=tj.device)
        gj = torch.empty(n, device=tj.device)
        gm = torch.empty(n, device=tj.device)
        call("hreg_js_loss", tj, tm, n, out, gj, gm, _stream())
        ctx.save_for_backward(gj, gm)
        return out[0]

    @staticmethod
    def backward(ctx, gout):
        gj, gm = ctx.saved_tensors
        n = gj.shape[0]
        s = gout.reshape(1).contiguous().float()
        dj = torch.empty_like(gj)
        dm = torch.empty_like(gm)
        # scale by the upstream gradient on the device (rowdot with C = 1)
        call("hreg_rowdot", gj, n, 1, s, None, 0, dj, _stream())
        call("hreg_rowdot", gm, n, 1, s, None, 0, dm, _stream())
        return dj, dm


def _conv_param(out_c, in_c, bias=False):
    w = torch.nn.Parameter(torch.empty(out_c, in_c, 1))
    torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5))
    b = None
    if bias:
        b = torch.nn.Parameter(torch.empty(out_c))
        torch.nn.init.uniform_(b, -1 / math.sqrt(in_c), 1 / math.sqrt(in_c))
    return w, b


class _Conv1x1(torch.nn.Module):
    """Parameter holder with nn.Conv1d(k=1, bias=False)'s names and shapes."""

    def __init__(self, in_c, out_c):
        super().__init__()
        self.weight, _ = _conv_param(out_c, in_c)


class _Lin(torch.nn.Module):
    """Parameter holder with nn.Linear's names and shapes."""

    def __init__(self, in_c, out_c):
        super().__init__()
        w, b = _conv_param(out_c, in_c, bias=True)
        self.weight = torch.nn.Parameter(w.detach().reshape(out_c, in_c))
        self.bias = b


class GlobalinfolossNet(torch.nn.Module):
    """mi_loss_v2.py:7-22: cat -> c1 (2C->C/2) -> c2 (C/4) -> c3 (C/8), ReLU each -> l0."""

    def __init__(self, in_channels: int):
        super().__init__()
        C = in_channels
        self.c1 = _Conv1x1(2 * C, C // 2)
        self.c2 = _Conv1x1(C // 2, C // 4)
        self.c3 = _Conv1x1(C // 4, C // 8)
        self.l0 = _Lin(C // 8, 1)

    def scores(self, rows: torch.Tensor) -> torch.Tensor:
        """rows [R, 2C] (already concatenated) -> [R]."""
        h = rows
        for conv in (self.c1, self.c2, self.c3):
            h = _LinearAct.apply(h, conv.weight.reshape(conv.weight.shape[0], -1), None, True)
        return _RowDot.apply(h, self.l0.weight.reshape(-1), self.l0.bias, False)

    def forward(self, x_global, c_global):
        return self.scores(torch.cat([_rows(x_global), _rows(c_global)], 1)).view(-1, 1)


class LocalinfolossNet(torch.nn.Module):
    """mi_loss_v2.py:25-39: cat -> conv1 (2C->C/2) -> conv2 (C/4) -> conv3 (1), ReLU each."""

    def __init__(self, in_channels: int):
        super().__init__()
        C = in_channels
        self.conv1 = _Conv1x1(2 * C, C // 2)
        self.conv2 = _Conv1x1(C // 2, C // 4)
        self.conv3 = _Conv1x1(C // 4, 1)

    def scores(self, rows: torch.Tensor) -> torch.Tensor:
        h = rows
        for conv in (self.conv1, self.conv2):
            h = _LinearAct.apply(h, conv.weight.reshape(conv.weight.shape[0], -1), None, True)
        return _RowDot.apply(h, self.conv3.weight.reshape(-1), None, True)

    def forward(self, x_local, c_local):
        """[B, C, N] x 2 -> [B, N]."""
        B, _, N = x_local.shape
        return self.scores(torch.cat([_rows(x_local), _rows(c_local)], 1)).view(B, N)


class DeepMILoss(torch.nn.Module):
    """mi_loss_v2.py:42-79.  As there, the discriminator is called as d(c, x): the
    context goes first in the channel concatenation."""

    def __init__(self, global_in_channels: int = None, local_in_channels: int = None):
        super().__init__()
        self.global_d = GlobalinfolossNet(global_in_channels) if global_in_channels else None
        self.local_d = LocalinfolossNet(local_in_channels) if local_in_channels else None
        if self.global_d is None and self.local_d is None:
            raise AttributeError("MI loss not found")

    @staticmethod
    def _js(d, c, x, x_prime):
        cr, xr, pr = _rows(c), _rows(x), _rows(x_prime)
        n = xr.shape[0]
        t = d.scores(torch.cat([torch.cat([cr, xr], 1), torch.cat([cr, pr], 1)], 0))
        return _JS.apply(t[:n], t[n:])

    def compute_local_loss(self, x_local, x_local_prime, c_local):
        return self._js(self.local_d, c_local, x_local, x_local_prime)

    def compute_global_loss(self, x_global, x_global_prime, c_global):
        return self._js(self.global_d, c_global, x_global, x_global_prime)

    def forward(self, x_global=None, x_global_prime=None, x_local=None, x_local_prime=None,
                c_local=None, c_global=None):
        total = 0
        if self.local_d is not None:
            total = total + self.compute_local_loss(x_local, x_local_prime, c_local)
        if self.global_d is not None:
            total = total + self.compute_global_loss(x_global, x_global_prime, c_global)
        return total


class ChamferDistanceLoss(torch.nn.Module):
    """losses/chamfer_loss.py:20-36 (forward; see the module docstring)."""

    def __init__(self, scale=1.0, reduction="mean"):
        super().__init__()
        assert reduction in ["sum", "mean", "none"], "Unknown or invalid reduction"
        self.reduction = reduction
        self.scale = scale

    def forward(self, template: torch.Tensor, source: torch.Tensor) -> torch.Tensor:
        if (template.dim() != 3 or source.dim() != 3 or template.shape[-1] != 3
                or source.shape[-1] != 3 or not template.is_cuda or not source.is_cuda):
            raise RuntimeError("ChamferDistanceLoss: [B, N, 3] GPU tensors expected "
                               "(there is no CPU fallback)")
        p0 = template.contiguous().float()
        p1 = source.contiguous().float()
        B, n, _ = p0.shape
        m = p1.shape[1]
        dev = p0.device
        d01 = torch.empty(B, n, device=dev)
        d10 = torch.empty(B, m, device=dev)
        per = torch.empty(B, device=dev)
        out = torch.empty(1, device=dev)
        red = {"none": _lib.HREG_REDUCE_NONE, "mean": _lib.HREG_REDUCE_MEAN,
               "sum": _lib.HREG_REDUCE_SUM}[self.reduction]
        call("hreg_chamfer", p0, p1, B, n, m, float(self.scale), red, d01, d10, None, None, per,
             out, _stream())
        return per if self.reduction == "none" else out[0]
