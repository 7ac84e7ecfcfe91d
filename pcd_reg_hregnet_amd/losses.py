"""Registration losses and metrics of the reference (losses/losses.py) on the HIP library.

transformation_loss keeps the reference's signature and 7-tuple result
(losses/losses.py:97-134); the per-pair work and the batch means run in one
kernel (csrc/losses.hip, hreg_transformation_loss).  Forward only: the
training backward is SURVEY.md 8(f) rank 1, not built yet.
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
