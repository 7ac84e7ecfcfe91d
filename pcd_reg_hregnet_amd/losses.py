"""Registration losses and metrics of the reference (losses/losses.py) on the HIP library.

transformation_loss keeps the reference's signature and 7-tuple result
(losses/losses.py:97-134); the per-pair work and the batch means run in one
kernel (csrc/losses.hip, hreg_transformation_loss).  As in the reference, loss,
loss_R and loss_t are differentiable in pred_R / pred_t when those require grad
(backward: hreg_transformation_loss_bwd through train_graph.transformation_loss);
the error metrics (R_err, geodesic_dist, T_err, eucl_dist) are returned without
gradient (the reference's trainers only log them).
"""
from __future__ import annotations

import torch

from . import _lib


def _check(t: torch.Tensor, name: str, shape) -> torch.Tensor:
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f"transformation_loss: {name} must be a GPU tensor (no CPU fallback)")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"transformation_loss: {name} has shape {tuple(t.shape)}, expected {shape}")
    return t.detach().float().contiguous()


def transformation_loss(pred_R, pred_t, gt_R, gt_t, alpha=1.0):
    """losses/losses.py:97-134.  pred_R/gt_R [B,3,3], pred_t/gt_t [B,3] ->
    (loss, loss_R, loss_t, R_err [3] deg, geodesic_dist [B] deg, T_err [3], eucl_dist [B])."""
    B = pred_R.shape[0]
    if B == 0:
        raise ValueError("transformation_loss: empty batch (the reference's mean would be NaN)")
    pR = _check(pred_R, "pred_R", (B, 3, 3))
    pt = _check(pred_t, "pred_t", (B, 3))
    gR = _check(gt_R, "gt_R", (B, 3, 3))
    gt = _check(gt_t, "gt_t", (B, 3))
    dev = pR.device
    scalars = torch.empty(3, device=dev)
    R_err = torch.empty(3, device=dev)
    T_err = torch.empty(3, device=dev)
    geo = torch.empty(B, device=dev)
    eucl = torch.empty(B, device=dev)
    _lib.call("hreg_transformation_loss", pR, pt, gR, gt, B, float(alpha), scalars, R_err, T_err,
              geo, eucl, _lib.stream_handle())
    if torch.is_grad_enabled() and (pred_R.requires_grad or pred_t.requires_grad):
        from . import train_graph
        R, t = pred_R.float().contiguous(), pred_t.float().contiguous()
        loss, _ = train_graph.transformation_loss(R, t, gR, gt, alpha)
        # loss_R / loss_t: the alpha = 1 loss with the other input detached carries
        # exactly the gradient of that part; its value is replaced by the part's
        lR = train_graph.transformation_loss(R, t.detach(), gR, gt, 1.0)[0]
        lt = train_graph.transformation_loss(R.detach(), t, gR, gt, 1.0)[0]
        return (loss, lR - lR.detach() + scalars[1], lt - lt.detach() + scalars[2], R_err, geo,
                T_err, eucl)
    return scalars[0], scalars[1], scalars[2], R_err, geo, T_err, eucl


def calc_rot_rre_err(pred_R, gt_R):
    """losses/losses.py:137-149 -> (mean |Euler XYZ| deg [3], geodesic deg [B])."""
    zeros = torch.zeros(pred_R.shape[0], 3, device=pred_R.device)
    out = transformation_loss(pred_R, zeros, gt_R, zeros)
    return out[3], out[4]


def calc_tran_rte_err(pred_t, gt_t):
    """losses/losses.py:151-160 -> (mean |dt| [3], ||dt|| [B])."""
    eye = torch.eye(3, device=pred_t.device).expand(pred_t.shape[0], 3, 3)
    out = transformation_loss(eye, pred_t, eye, gt_t)
    return out[5], out[6]
