"""Drop-in for the reference's pybind module ``point_utils_cuda``.

Same four functions, argument order and meaning as
models/PointUtils/src/point_utils_api.cpp:6-12 (prototypes
furthest_point_sampling_gpu.h:8-30): the caller allocates every tensor,
work is enqueued on the current stream, the call returns 1.  Unlike the
reference (which prints and calls exit(-1) on a launch error,
furthest_point_sampling_gpu.cu:35-38) errors raise RuntimeError.
Backed by libhregnet_amd.so (gfx950); there is no CPU path.
"""
from __future__ import annotations

import torch

from . import _lib


def _check(t: torch.Tensor, name: str, dtype) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a GPU tensor")
    if t.dtype != dtype:
        raise RuntimeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")


def furthest_point_sampling_wrapper(b: int, n: int, m: int, points_tensor: torch.Tensor,
                                    temp_tensor: torch.Tensor, idx_tensor: torch.Tensor) -> int:
    """furthest_point_sampling.cpp:33-43"""
    _check(points_tensor, "points", torch.float32)
    _check(temp_tensor, "temp", torch.float32)
    _check(idx_tensor, "idx", torch.int32)
    _lib.call("hreg_furthest_point_sampling", b, n, m, points_tensor, temp_tensor, idx_tensor,
              None, _lib.stream_handle())
    return 1


def weighted_furthest_point_sampling_wrapper(b: int, n: int, m: int, points_tensor: torch.Tensor,
                                             weights_tensor: torch.Tensor,
                                             temp_tensor: torch.Tensor,
                                             idx_tensor: torch.Tensor) -> int:
    """furthest_point_sampling.cpp:45-55"""
    _check(points_tensor, "points", torch.float32)
    _check(weights_tensor, "weights", torch.float32)
    _check(temp_tensor, "temp", torch.float32)
    _check(idx_tensor, "idx", torch.int32)
    _lib.call("hreg_weighted_furthest_point_sampling", b, n, m, points_tensor, weights_tensor,
              temp_tensor, idx_tensor, None, _lib.stream_handle())
    return 1


def gather_points_wrapper(b: int, c: int, n: int, npoints: int, points_tensor: torch.Tensor,
                          idx_tensor: torch.Tensor, out_tensor: torch.Tensor) -> int:
    """furthest_point_sampling.cpp:10-19"""
    _check(points_tensor, "points", torch.float32)
    _check(idx_tensor, "idx", torch.int32)
    _check(out_tensor, "out", torch.float32)
    _lib.call("hreg_gather_points", b, c, n, npoints, points_tensor, idx_tensor, out_tensor,
              _lib.stream_handle())
    return 1


def gather_points_grad_wrapper(b: int, c: int, n: int, npoints: int,
                               grad_out_tensor: torch.Tensor, idx_tensor: torch.Tensor,
                               grad_points_tensor: torch.Tensor) -> int:
    """furthest_point_sampling.cpp:21-31"""
    _check(grad_out_tensor, "grad_out", torch.float32)
    _check(idx_tensor, "idx", torch.int32)
    _check(grad_points_tensor, "grad_points", torch.float32)
    _lib.call("hreg_gather_points_grad", b, c, n, npoints, grad_out_tensor, idx_tensor,
              grad_points_tensor, _lib.stream_handle())
    return 1
