"""Point-to-point ICP refinement after the network (reference test/test_v4.py:140-158).

The reference refines the finest predicted pose with open3d:

    reg_icp = o3d.pipelines.registration.registration_icp(
        source=src_pcd, target=dst_pcd, max_correspondence_distance=1.0, init=tf_init,
        estimation_method=TransformationEstimationPointToPoint(),
        criteria=ICPConvergenceCriteria(relative_fitness=1e-6, relative_rmse=1e-6,
                                        max_iteration=2000))
    pred_tf_4 = reg_icp.transformation

``registration_icp`` here is that call on the GPU for a whole batch of pairs
(csrc/icp.hip): the clouds stay in HBM, every iteration (spatially indexed nearest
neighbours within the distance, fp64 Kabsch update, convergence test) runs on the device,
and the host only polls the per-pair done flags every ``poll`` iterations.  open3d itself is
not installed here: its published loop is restated (parity unpinned against open3d; pinned
against oracle/oracle.py's CPU restatement and planted-transform tests).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import _lib


@dataclass
class ICPConvergenceCriteria:
    """open3d.pipelines.registration.ICPConvergenceCriteria (defaults as open3d's)."""
    relative_fitness: float = 1e-6
    relative_rmse: float = 1e-6
    max_iteration: int = 30


@dataclass
class RegistrationResult:
    """open3d RegistrationResult, batched: transformation [B,4,4], fitness [B],
    inlier_rmse [B]; iterations [B] = Kabsch updates applied."""
    transformation: torch.Tensor
    fitness: torch.Tensor
    inlier_rmse: torch.Tensor
    iterations: torch.Tensor


def registration_icp(source, target, max_correspondence_distance: float, init=None,
                     criteria: ICPConvergenceCriteria | None = None, poll: int = 8):
    """source [N,3] / [B,N,3], target [M,3] / [B,M,3] (fp32 on the GPU), init [4,4] /
    [B,4,4] (default identity) -> RegistrationResult (batched like the inputs)."""
    crit = criteria or ICPConvergenceCriteria()
    single = source.dim() == 2
    src = (source[None] if single else source).float().contiguous()
    dst = (target[None] if target.dim() == 2 else target).float().contiguous()
    B, ns, _ = src.shape
    nt = dst.shape[1]
    if dst.shape[0] != B:
        raise ValueError("source and target batch sizes differ")
    dev = src.device
    T0 = None
    if init is not None:
        T0 = torch.as_tensor(init, dtype=torch.float32, device=dev)
        T0 = (T0[None] if T0.dim() == 2 else T0).expand(B, 4, 4).contiguous()
    L = _lib.load()
    ws = torch.empty(L.hreg_icp_ws_bytes(B, ns, nt) + 256, dtype=torch.uint8, device=dev)
    off = (-ws.data_ptr()) % 256
    wsp = ws[off:]
    st = _lib.stream_handle()
    _lib.call("hreg_icp_init", src, dst, B, ns, nt, T0, wsp, st)
    T = torch.empty(B, 4, 4, device=dev)
    fit = torch.empty(B, device=dev)
    rmse = torch.empty(B, device=dev)
    its = torch.empty(B, dtype=torch.int32, device=dev)
    done = torch.empty(B, dtype=torch.int32, device=dev)
    # max_iteration updates need max_iteration + 1 correspondence passes
    left = crit.max_iteration + 1
    while left > 0:
        n = min(poll, left)
        _lib.call("hreg_icp_iterate", dst, B, ns, nt, float(max_correspondence_distance),
                  float(crit.relative_fitness), float(crit.relative_rmse), int(crit.max_iteration),
                  n, wsp, st)
        left -= n
        _lib.call("hreg_icp_result", wsp, B, ns, nt, None, None, None, None, done, st)
        if bool(done.all()):  # one sync per `poll` iterations
            break
    _lib.call("hreg_icp_result", wsp, B, ns, nt, T, fit, rmse, its, done, st)
    if single:
        return RegistrationResult(T[0], fit[0], rmse[0], its[0])
    return RegistrationResult(T, fit, rmse, its)
