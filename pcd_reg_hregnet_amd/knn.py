"""Drop-in for ``pytorch3d.ops.knn_points`` / ``knn_gather`` as HRegNet calls them.

Reference dependency: pytorch3d 0.7.8 (Dockerfile:44-46), not vendored; call
sites models/HRegNet/layers.py:20,25,278-279,288,303,309,316-317,322-323,352,
358,434,437,443.  Returns squared L2 distances sorted ascending with the
canonical (dist, idx) tie order (pytorch3d sorts with an unstable torch.sort:
its tie order is parity unpinned).  K <= 64 (the kernel's register list; HRegNet's
largest K is 64).  Heterogeneous ``lengths`` (r6; HRegNet never passes them): cloud b's
p1 rows i >= lengths1[b] and neighbour slots beyond lengths2[b] are padding, returned as
dist 0 / idx -1 (the library's k > n2 convention) -- pytorch3d's padding values are not
in this image, so that part is parity unpinned; the valid rows are the same kernel's
selections over the cloud's first lengths2[b] points.  knn_gather(lengths) zeroes the
slots k >= lengths[b] as pytorch3d's does.
"""
from __future__ import annotations

from collections import namedtuple

import torch
from torch.autograd import Function

from . import _lib

_KNN = namedtuple("KNN", "dists idx knn")


def _lengths(lengths, B: int, N: int, name: str):
    """host list of per-cloud lengths (None: all N), checked against [0, N]"""
    if lengths is None:
        return [N] * B
    ls = [int(v) for v in torch.as_tensor(lengths).reshape(-1).tolist()]
    if len(ls) != B or any(v < 0 or v > N for v in ls):
        raise ValueError(f"knn_points: {name} must hold {B} lengths in [0, {N}]")
    return ls


def knn_points(p1: torch.Tensor, p2: torch.Tensor, lengths1=None, lengths2=None, norm: int = 2,
               K: int = 1, version: int = -1, return_nn: bool = False,
               return_sorted: bool = True):
    if norm != 2:
        raise NotImplementedError("knn_points: only squared L2 (norm=2)")
    if p1.shape[0] != p2.shape[0] or p1.shape[2] != p2.shape[2]:
        raise ValueError("pts1 and pts2 must have the same batch and point dimension")
    p1c = p1.detach().float().contiguous()
    p2c = p2.detach().float().contiguous()
    B, N1, D = p1c.shape
    N2 = p2c.shape[1]
    st = _lib.stream_handle()
    if lengths1 is None and lengths2 is None:
        dists = torch.empty((B, N1, K), dtype=torch.float32, device=p1.device)
        idx = torch.empty((B, N1, K), dtype=torch.int64, device=p1.device)
        _lib.call("hreg_knn_points", p1c, p2c, B, N1, N2, D, K, dists, idx, None, None, st)
    else:
        # ragged clouds: one launch per cloud over its valid rows / points (a compatibility
        # path: HRegNet's own calls are dense)
        l1, l2 = _lengths(lengths1, B, N1, "lengths1"), _lengths(lengths2, B, N2, "lengths2")
        dists = torch.zeros((B, N1, K), dtype=torch.float32, device=p1.device)
        idx = torch.full((B, N1, K), -1, dtype=torch.int64, device=p1.device)
        for b in range(B):
            if l1[b] == 0 or l2[b] == 0:
                continue
            d_b = torch.empty((1, l1[b], K), dtype=torch.float32, device=p1.device)
            i_b = torch.empty((1, l1[b], K), dtype=torch.int64, device=p1.device)
            _lib.call("hreg_knn_points", p1c[b:b + 1, :l1[b]].contiguous(), p2c[b:b + 1, :l2[b]].contiguous(),
                      1, l1[b], l2[b], D, K, d_b, i_b, None, None, st)
            dists[b, :l1[b]] = d_b[0]
            idx[b, :l1[b]] = i_b[0]
    nn = knn_gather(p2, idx, lengths2) if return_nn else None
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
    """x [B,N,C], idx [B,M,K] -> [B,M,K,C] (differentiable in x).  lengths [B]: the slots
    k >= lengths[b] gather zeros (pytorch3d's mask; here by idx -1, which the gather kernel
    reads as a zero row and the backward discards)."""
    if lengths is not None:
        B, _, K = idx.shape
        ls = torch.as_tensor(lengths, device=idx.device).reshape(B, 1, 1)
        keep = torch.arange(K, device=idx.device).view(1, 1, K) < ls
        idx = torch.where(keep, idx, torch.full_like(idx, -1))
    return _KnnGather.apply(x, idx)
