"""Drop-in for ``pytorch3d.ops.knn_points`` / ``knn_gather`` as HRegNet calls them.

Reference dependency: pytorch3d 0.7.8 (Dockerfile:44-46), not vendored; call
sites models/HRegNet/layers.py:20,25,278-279,288,303,309,316-317,322-323,352,
358,434,437,443.  Returns squared L2 distances sorted ascending with the
canonical (dist, idx) tie order (pytorch3d sorts with an unstable torch.sort:
its tie order is parity unpinned).  K <= 64, heterogeneous ``lengths`` are not
supported (HRegNet never passes them).
"""
from __future__ import annotations

from collections import namedtuple

import torch
from torch.autograd import Function

from . import _lib

_KNN = namedtuple("KNN", "dists idx knn")


def knn_points(p1: torch.Tensor, p2: torch.Tensor, lengths1=None, lengths2=None, norm: int = 2,
               K: int = 1, version: int = -1, return_nn: bool = False,
               return_sorted: bool = True):
    if lengths1 is not None or lengths2 is not None:
        raise NotImplementedError("knn_points: per-cloud lengths are not supported")
    if norm != 2:
        raise NotImplementedError("knn_points: only squared L2 (norm=2)")
    if p1.shape[0] != p2.shape[0] or p1.shape[2] != p2.shape[2]:
        raise ValueError("pts1 and pts2 must have the same batch and point dimension")
    p1c = p1.detach().float().contiguous()
    p2c = p2.detach().float().contiguous()
    B, N1, D = p1c.shape
    N2 = p2c.shape[1]
    dists = torch.empty((B, N1, K), dtype=torch.float32, device=p1.device)
    idx = torch.empty((B, N1, K), dtype=torch.int64, device=p1.device)
    _lib.call("hreg_knn_points", p1c, p2c, B, N1, N2, D, K, dists, idx, None, None,
              _lib.stream_handle())
    nn = knn_gather(p2, idx) if return_nn else None
    return _KNN(dists=dists, idx=idx, knn=nn)


class _KnnGather(Function):
    @staticmethod
    def forward(ctx, x, idx):
        B, N, C = x.shape
        _, M, K = idx.shape
        xc = x.contiguous().float()
        ic = idx.contiguous().long()
        out = torch.empty((B, M, K, C), dtype=torch.float32, device=x.device)
        _lib.call("hreg_knn_gather", xc, ic, B, N, C, M, K, out, _lib.stream_handle())
        ctx.save_for_backward(ic)
        ctx.N = N
        return out

    @staticmethod
    def backward(ctx, grad):
        """dx[b, n] = sum of grad[b, m, k] over the (m, k) with idx[b, m, k] == n, summed in
        ascending (m, k) order by the library's CSR scatter (hreg_csr_build +
        hreg_scatter_rows: deterministic, no atomics); padded entries (idx < 0) go to a
        discarded row (out-of-range entries gather zeros in the forward)."""
        (idx,) = ctx.saved_tensors
        B, M, K = idx.shape
        C = grad.shape[-1]
        N = ctx.N
        n = B * N + 1                                   # + the row that takes idx < 0
        rows = idx + torch.arange(B, device=idx.device).view(B, 1, 1) * N
        gi = torch.where((idx >= 0) & (idx < N), rows, torch.full_like(rows, n - 1)).to(torch.int32)
        gi = gi.reshape(-1).contiguous()
        Mt = gi.numel()
        st = _lib.stream_handle()
        ws = torch.empty(max(int(_lib.load().hreg_csr_ws_bytes(Mt, n)), 16), dtype=torch.uint8,
                         device=grad.device)
        _lib.call("hreg_csr_build", gi, Mt, n, ws, st)
        dy = grad.float().contiguous().view(Mt, C)
        dx = torch.empty((n, C), dtype=torch.float32, device=grad.device)
        _lib.call("hreg_scatter_rows", dy, C, ws, Mt, n, C, dx, C, 0, st)
        return dx[:B * N].view(B, N, C).to(grad.dtype), None


def knn_gather(x: torch.Tensor, idx: torch.Tensor, lengths=None):
    """x [B,N,C], idx [B,M,K] -> [B,M,K,C] (differentiable in x)."""
    if lengths is not None:
        raise NotImplementedError("knn_gather: lengths are not supported")
    return _KnnGather.apply(x, idx)
