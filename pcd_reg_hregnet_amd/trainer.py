"""HRegNet training step (BASELINE configs[3]: train_reg_v0, batch sharded over ranks).

One step of train/train_reg_v0.py:264-294 -- ``optimizer.zero_grad()``, the train-mode
forward, l_trans = mean over the 3 levels of ``transformation_loss`` (alpha), backward,
``optimizer.step()`` (Adam, train_reg_v0.py:249) -- restated for one process per GPU:

* parameters and their gradients live in two flat fp32 buffers (2,467,846 floats for
  HRegNet, SURVEY.md 8(e), each tensor 256-byte aligned); every ``p`` / ``p.grad`` is a
  view into them, so the backward writes straight into the gradient bucket;
* with ``torch.distributed`` initialised (RCCL over xGMI on the GPU box), the bucket is
  averaged with ONE all_reduce per step (a 9.87 MB ring pass, not one collective per
  tensor), which is DistributedDataParallel's gradient semantics; ranks start from
  rank 0's parameters (one broadcast at construction);
* Adam is one launch over the flat buffers (csrc/train.hip ``adam_kernel``, the same
  arithmetic as torch.optim.Adam's foreach path);
* BatchNorm statistics are per rank (the reference does not use SyncBN).

``StepLR(step_size=10, gamma=0.5)`` (train_reg_v0.py:250) is per epoch: ``set_lr``.
"""
from __future__ import annotations

import weakref

import torch
import torch.distributed as dist

from . import _lib, engine, train_graph
from .train import GradBucket, flat_offsets


def _dist_world(group=None) -> int:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group)
    return 1


class FlatParams:
    """Re-home every trainable parameter into one flat buffer (p.data becomes a view)."""

    def __init__(self, params):
        self.params = [p for p in params if p.requires_grad]
        offs, n = flat_offsets(self.params)
        self.flat = torch.zeros(n, dtype=torch.float32, device=self.params[0].device)
        for p, off in zip(self.params, offs):
            k = p.numel()
            self.flat[off:off + k].copy_(p.detach().reshape(-1))
            p.data = self.flat[off:off + k].view_as(p)

    def broadcast(self, src: int = 0, group=None):
        if _dist_world(group) > 1:
            dist.broadcast(self.flat, src=src, group=group)


class FlatAdam:
    """torch.optim.Adam over the flat parameter / gradient buffers: one launch per step."""

    def __init__(self, flat_params: FlatParams, bucket: GradBucket, lr=1e-3,
                 betas=(0.9, 0.999), eps=1e-8):
        self.p = flat_params.flat
        self.g = bucket.flat
        assert self.p.numel() == self.g.numel()
        self.m = torch.zeros_like(self.p)
        self.v = torch.zeros_like(self.p)
        self.lr, self.betas, self.eps = lr, betas, eps
        self.step_count = 0

    @torch.no_grad()
    def step(self):
        self.step_count += 1
        _lib.call("hreg_adam_step", self.p, self.g, self.m, self.v, self.p.numel(),
                  float(self.lr), float(self.betas[0]), float(self.betas[1]), float(self.eps),
                  self.step_count, _lib.stream_handle())


class Level1Prefetch:
    """Level-1 FPS + kNN grouping of a batch (input-only, weight-independent: the same
    selections whenever they are computed) for src and dst in one launch set, on a side
    stream.  The trainer starts it for batch i+1 before running step i, so the level-1
    FPS (one workgroup per cloud, ~1.8 ms at N = 16384) runs beside step i's kernels.

    A prefetch belongs to the exact tensor objects it was started on, at their version
    counters of that moment: ``take`` matches on weak references to src / dst (a freed
    tensor whose address the caching allocator hands out again is a different object)
    and on ``Tensor._version`` (a static buffer refilled in place with ``copy_`` bumps
    it), so a step never runs on selections computed from other contents.  Writes that
    bypass autograd's version counter (a raw-pointer kernel filling the buffer) are not
    seen: pass a fresh tensor, or call ``discard()``, after such a write."""

    def __init__(self, device):
        self.stream = torch.cuda.Stream(device=device)
        self.key = None
        self.prepared = None
        self.event = None

    def start(self, src, dst):
        main = torch.cuda.current_stream()
        self.stream.wait_stream(main)  # src / dst are written on the main stream
        with torch.cuda.stream(self.stream):
            B, n, _ = src.shape
            M, k = engine.LEVELS[0][:2]
            pts = torch.cat([src, dst], 0)
            idx, _, gidx, _, _ = engine.grouping(pts, 0)
            src_fps, dst_fps = idx[:B], idx[B:]
            prepared = {
                "src_fps_1": (src_fps, train_graph.offset_index(src_fps, n)),
                "dst_fps_1": (dst_fps, train_graph.offset_index(dst_fps, n)),
                "src_knn_1": (None, gidx[:B * M * k]),
                "dst_knn_1": (None, (gidx[B * M * k:] - B * n).to(torch.int32)),
            }
            self.event = torch.cuda.Event()
            self.event.record(self.stream)
        for loc, g in prepared.values():
            for t in (loc, g):
                if t is not None:
                    t.record_stream(main)  # consumed on the main stream
        self.key = self._key(src, dst)
        self.prepared = prepared

    @staticmethod
    def _key(src, dst):
        return (weakref.ref(src), weakref.ref(dst), src._version, dst._version,
                src.data_ptr(), dst.data_ptr(), tuple(src.shape))

    def matches(self, src, dst) -> bool:
        if self.key is None:
            return False
        rs, rd, vs, vd, ps, pd, shape = self.key
        return (rs() is src and rd() is dst and src._version == vs and dst._version == vd
                and (src.data_ptr(), dst.data_ptr(), tuple(src.shape)) == (ps, pd, shape))

    def discard(self):
        self.key, self.prepared = None, None

    def take(self, src, dst):
        """The prefetched selections if they belong to (src, dst) as they were when the
        prefetch started, else None (and the stale prefetch is dropped)."""
        if not self.matches(src, dst):
            self.discard()
            return None
        torch.cuda.current_stream().wait_event(self.event)
        prepared = self.prepared
        self.discard()
        return prepared


class Trainer:
    """``step(src, dst, gt_R, gt_t)`` = one train_reg_v0 iteration on this rank's shard.
    ``next_batch=(src, dst)`` starts the next batch's level-1 grouping on a side stream."""

    def __init__(self, net, lr=1e-3, alpha=1.0, group=None):
        self.net = net.train()
        self.alpha = alpha
        self.group = group
        self.params = FlatParams(net.parameters())
        self.params.broadcast(0, group)
        self.bucket = GradBucket(self.params.params)
        self.opt = FlatAdam(self.params, self.bucket, lr=lr)
        self.prefetch = Level1Prefetch(self.params.flat.device)

    def set_lr(self, lr: float):
        self.opt.lr = lr

    def step(self, src, dst, gt_R, gt_t, next_batch=None):
        """-> (loss, l_R, l_t) of this rank's shard (detached, on the device)."""
        prepared = self.prefetch.take(src, dst)
        # FPS only: with use_fps=False the level-1 sample is a host RNG draw made in the
        # forward, in the reference's order
        if next_batch is not None and self.net.feature_extraction.use_fps:
            self.prefetch.start(*next_batch)
        self.bucket.attach()                     # optimizer.zero_grad()
        hook = train_graph.IndexHook(prepared=prepared) if prepared else None
        ret = train_graph.hregnet_train_forward(self.net, src, dst, hook)
        loss, l_R, l_t = train_graph.registration_loss(ret, gt_R, gt_t, self.alpha)
        loss.backward()
        self.bucket.collect()
        self.bucket.all_reduce_mean(self.group)  # DDP gradient averaging, one collective
        self.opt.step()
        return loss.detach(), l_R.detach(), l_t.detach()
