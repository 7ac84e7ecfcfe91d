"""Autograd op wrappers -- drop-in for the reference's models/utils.py:14-89.

``furthest_point_sample``, ``weighted_furthest_point_sample`` and
``gather_operation`` keep the reference names, arguments and outputs; they run
on the HIP library through :mod:`point_utils_cuda`.  Buffers are allocated on
the input's device (the reference uses torch.cuda.IntTensor/FloatTensor,
models/utils.py:24-25, 48-49, 73, 84).
"""
from __future__ import annotations

import random

import numpy as np
import torch
from torch.autograd import Function

from . import point_utils_cuda


class FurthestPointSampling(Function):
    """models/utils.py:14-34"""

    @staticmethod
    def forward(ctx, xyz: torch.Tensor, npoint: int) -> torch.Tensor:
        assert xyz.is_contiguous()
        B, N, _ = xyz.size()
        output = torch.empty((B, npoint), dtype=torch.int32, device=xyz.device)
        temp = torch.full((B, N), 1e10, dtype=torch.float32, device=xyz.device)
        point_utils_cuda.furthest_point_sampling_wrapper(B, N, npoint, xyz, temp, output)
        return output

    @staticmethod
    def backward(ctx, a=None):
        return None, None


furthest_point_sample = FurthestPointSampling.apply


class WeightedFurthestPointSampling(Function):
    """models/utils.py:36-58"""

    @staticmethod
    def forward(ctx, xyz: torch.Tensor, weights: torch.Tensor, npoint: int) -> torch.Tensor:
        assert xyz.is_contiguous()
        assert weights.is_contiguous()
        B, N, _ = xyz.size()
        output = torch.empty((B, npoint), dtype=torch.int32, device=xyz.device)
        temp = torch.full((B, N), 1e10, dtype=torch.float32, device=xyz.device)
        point_utils_cuda.weighted_furthest_point_sampling_wrapper(B, N, npoint, xyz, weights, temp,
                                                                  output)
        return output

    @staticmethod
    def backward(ctx, a=None):
        return None, None, None


weighted_furthest_point_sample = WeightedFurthestPointSampling.apply


class GatherOperation(Function):
    """models/utils.py:60-89: out[b,c,j] = features[b,c,idx[b,j]]; grad scatter-adds."""

    @staticmethod
    def forward(ctx, features: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
        assert features.is_contiguous()
        assert idx.is_contiguous()
        B, npoint = idx.size()
        _, C, N = features.size()
        output = torch.empty((B, C, npoint), dtype=torch.float32, device=features.device)
        point_utils_cuda.gather_points_wrapper(B, C, N, npoint, features, idx, output)
        ctx.for_backwards = (idx, C, N)
        return output

    @staticmethod
    def backward(ctx, grad_out):
        idx, C, N = ctx.for_backwards
        B, npoint = idx.size()
        grad_features = torch.zeros((B, C, N), dtype=torch.float32, device=grad_out.device)
        point_utils_cuda.gather_points_grad_wrapper(B, C, N, npoint, grad_out.contiguous(), idx,
                                                    grad_features)
        return grad_features, None


gather_operation = GatherOperation.apply


def set_seed(seed):
    """models/utils.py:140-152"""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
        torch.cuda.manual_seed_all(seed)
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = True


def calc_error_np(pred_R, pred_t, gt_R, gt_t):
    """models/utils.py:132-138: rotation error (deg) and translation error (m)."""
    tmp = (np.trace(pred_R.transpose().dot(gt_R)) - 1) / 2
    tmp = np.clip(tmp, -1.0, 1.0)
    L_rot = 180 * np.arccos(tmp) / np.pi
    L_trans = np.linalg.norm(pred_t - gt_t)
    return L_rot, L_trans
