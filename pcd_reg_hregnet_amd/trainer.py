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

import math
import weakref

import numpy as np
import torch
import torch.distributed as dist

from . import _lib, capture, engine, train_graph
from .train import GradBucket, flat_offsets


# src and dst feature extraction (and their backwards) on two streams
# (train_graph.hregnet_train_forward(concurrent=True)): the same results as the serial step
TWO_STREAM = True


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
        # (no side stream for a CPU trainer: the host-logic tests build one around stubs)
        self.stream = torch.cuda.Stream(device=device) if torch.device(device).type == "cuda" else None
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


def ddp_average(bucket: GradBucket, group=None, force: bool = False) -> None:
    """DistributedDataParallel's gradient averaging for one step: ONE all_reduce (SUM) of the
    whole flat bucket (every parameter's gradient in FlatParams order), then / world -- a no-op
    in a single process unless ``force`` (Trainer(always_reduce=True): the collective runs at
    world 1 too, so the captured RCCL node is exercised on a one-GPU box).  Trainer.step and
    the captured GraphTrainer step both call exactly this (tests/test_distributed.py counts the
    collectives of a real Trainer.step on gloo)."""
    bucket.all_reduce_mean(group, force=force)


class Trainer:
    """``step(src, dst, gt_R, gt_t)`` = one train_reg_v0 iteration on this rank's shard.
    ``next_batch=(src, dst)`` starts the next batch's level-1 grouping on a side stream."""

    def __init__(self, net, lr=1e-3, alpha=1.0, group=None, always_reduce: bool = False):
        self.net = net.train()
        self.alpha = alpha
        self.group = group
        # issue the bucket all-reduce even in a 1-rank process group (tests: the RCCL node of
        # the captured step on a one-GPU box); the sum over one rank / 1 is the identity
        self.always_reduce = always_reduce
        self.params = FlatParams(net.parameters())
        self.params.broadcast(0, group)
        self.bucket = GradBucket(self.params.params, sides=2)
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
        hook = train_graph.IndexHook(prepared=prepared) if prepared else None
        out = self.local_gradients(src, dst, gt_R, gt_t, hook)
        ddp_average(self.bucket, self.group, force=self.always_reduce)
        self.opt.step()
        return out

    def local_gradients(self, src, dst, gt_R, gt_t, hook=None):
        """This rank's half of a step: ``optimizer.zero_grad()``, the train-mode forward on
        the shard (BN statistics of the shard alone, running stats updated), the loss and its
        backward into the gradient bucket -- everything before DDP's all-reduce.  hook: an
        IndexHook (prepared / injected selections).  -> (loss, l_R, l_t), detached."""
        self.bucket.attach()                     # optimizer.zero_grad()
        try:
            two = TWO_STREAM and src.is_cuda
            ret = train_graph.hregnet_train_forward(self.net, src, dst, hook, concurrent=two)
            loss, l_R, l_t = train_graph.registration_loss(ret, gt_R, gt_t, self.alpha)
            loss.backward()
            if two:
                train_graph.join_side_stream(src.device)
            self.bucket.collect(two_sides=two)
        finally:
            GradBucket.direct_off()
        return loss.detach(), l_R.detach(), l_t.detach()


def level1_selections(src, dst):
    """The weight-independent level-1 selections of a batch (FPS + kNN grouping of src and dst
    in one launch set) in the IndexHook ``prepared`` form (Level1Prefetch's)."""
    B, n, _ = src.shape
    M, k = engine.LEVELS[0][:2]
    idx, _, gidx, _, _ = engine.grouping(torch.cat([src, dst], 0), 0)
    src_fps, dst_fps = idx[:B], idx[B:]
    return {
        "src_fps_1": (src_fps, train_graph.offset_index(src_fps, n)),
        "dst_fps_1": (dst_fps, train_graph.offset_index(dst_fps, n)),
        "src_knn_1": (None, gidx[:B * M * k]),
        "dst_knn_1": (None, (gidx[B * M * k:] - B * n).to(torch.int32)),
    }


class GraphTrainer:
    """``Trainer.step`` replayed from two captured HIP graphs (the step's
    ~1,500 launches and their host gaps).  Two static input sets ping-pong: replay i runs the
    step on set k = i % 2 with the level-1 selections the previous replay computed for it, and,
    on a side stream inside the same graph, the selections of set 1 - k (the next batch, copied
    in before the replay) -- Level1Prefetch's overlap, captured.  Adam reads its step's bias
    corrections from device memory (hreg_adam_step_dev), written before each replay, so lr
    changes (``set_lr``) need no recapture.  Everything else a step does -- BN running stats,
    num_batches_tracked, the gradient bucket -- is device work in the graph; with world > 1
    (RCCL) the bucket's one all-reduce is captured too (a graph node between the backward and
    Adam: ``ddp_average``, the same call the eager Trainer makes; the two eager warm-up steps
    before the capture initialise the communicator).  Capture runs two warm-up steps first; the
    parameters, optimizer moments and BN buffers are restored afterwards, so the first
    ``step`` continues from the state the Trainer had."""

    def __init__(self, trainer: "Trainer", batch: int, points: int):
        self.world = _dist_world(trainer.group)
        collective = self.world > 1 or (trainer.always_reduce and dist.is_available()
                                        and dist.is_initialized())
        if collective and dist.get_backend(trainer.group) != "nccl":
            # RCCL collectives are captured into the graph (the bucket all-reduce is a graph
            # node on the step's stream); gloo's host-side collectives cannot be
            raise NotImplementedError("GraphTrainer with world > 1 needs the nccl (RCCL) backend; "
                                      "with gloo use Trainer")
        if not trainer.net.feature_extraction.use_fps:
            # use_fps=False (layers.py:144-147) draws torch.randperm samples on the host per
            # step; a captured graph would freeze one draw and replay it forever
            raise NotImplementedError("GraphTrainer needs use_fps=True (random sampling draws "
                                      "on the host every step: use Trainer)")
        self.tr = trainer
        dev = trainer.params.flat.device
        self.src = [torch.zeros(batch, points, 3, device=dev) for _ in range(2)]
        self.dst = [torch.zeros(batch, points, 3, device=dev) for _ in range(2)]
        self.gR = [torch.eye(3, device=dev).repeat(batch, 1, 1) for _ in range(2)]
        self.gt = [torch.zeros(batch, 3, device=dev) for _ in range(2)]
        self.scal = torch.zeros(2, device=dev)
        # two pinned staging slots: a slot is rewritten only after its previous asynchronous
        # copy ran (its event), so a host running ahead never changes a pending step's scalars
        self.scal_h = [torch.zeros(2, pin_memory=True) for _ in range(2)]
        self.scal_ev = [None, None]
        self.scal_slot = 0
        self.side = torch.cuda.Stream(device=dev)
        self.sel = [None, None]
        self.graphs = [None, None]
        self.outs = [None, None]
        self.k = 0
        self.loaded = False

    def _sel_into(self, k):
        fresh = level1_selections(self.src[k], self.dst[k])
        if self.sel[k] is None:
            self.sel[k] = {nm: (None if a is None else a.clone(), b.clone()) for nm, (a, b) in fresh.items()}
            return
        for nm, (a, b) in fresh.items():
            sa, sb = self.sel[k][nm]
            if a is not None:
                sa.copy_(a)
            sb.copy_(b)

    def _set_scalars(self):
        """hreg_adam_step's bias corrections for the next step, with its arithmetic: lr and the
        betas as the fp32 kernel arguments, powers and quotient in double, rounded to fp32"""
        opt = self.tr.opt
        t = opt.step_count + 1
        f32 = lambda x: float(np.float32(x))  # noqa: E731
        lr, b1, b2 = f32(opt.lr), f32(opt.betas[0]), f32(opt.betas[1])
        i = self.scal_slot
        self.scal_slot ^= 1
        if self.scal_ev[i] is not None:
            self.scal_ev[i].synchronize()
        h = self.scal_h[i]
        h[0] = f32(lr / (1.0 - math.pow(b1, t)))
        h[1] = f32(math.sqrt(1.0 - math.pow(b2, t)))
        self.scal.copy_(h, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.scal_ev[i] = ev

    def _body(self, k):
        tr = self.tr
        cur = torch.cuda.current_stream()
        self.side.wait_stream(cur)  # the next set was copied in on this stream
        with torch.cuda.stream(self.side):
            self._sel_into(1 - k)
        tr.bucket.attach()
        try:
            hook = train_graph.IndexHook(prepared=self.sel[k])
            two = TWO_STREAM
            ret = train_graph.hregnet_train_forward(tr.net, self.src[k], self.dst[k], hook,
                                                    concurrent=two)
            loss, l_R, l_t = train_graph.registration_loss(ret, self.gR[k], self.gt[k], tr.alpha)
            loss.backward()
            if two:
                train_graph.join_side_stream(self.src[k].device)
            tr.bucket.collect(two_sides=two)
        finally:
            GradBucket.direct_off()
        # world > 1 (or always_reduce): the RCCL all-reduce, captured
        ddp_average(tr.bucket, tr.group, force=tr.always_reduce)
        opt = tr.opt
        _lib.call("hreg_adam_step_dev", opt.p, opt.g, opt.m, opt.v, opt.p.numel(), float(opt.lr),
                  float(opt.betas[0]), float(opt.betas[1]), float(opt.eps), self.scal,
                  _lib.stream_handle())
        cur.wait_stream(self.side)
        return loss.detach(), l_R.detach(), l_t.detach()

    def _state(self):
        tr = self.tr
        bufs = [b for b in tr.net.buffers()]
        return [tr.params.flat, tr.opt.m, tr.opt.v] + bufs

    def capture(self, src, dst, gt_R, gt_t):
        """Warm up and capture both graphs on this batch; the trainer's state is restored."""
        tr = self.tr
        saved = [t.detach().clone() for t in self._state()]
        step_count = tr.opt.step_count
        for k in (0, 1):
            self._load(k, src, dst, gt_R, gt_t)
        self._sel_into(0)
        s = torch.cuda.Stream(device=self.scal.device)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for k in (0, 1):  # eager warm-up of the exact bodies (allocator, lazy builds)
                self._set_scalars()
                self._body(k)
                tr.opt.step_count += 1
        torch.cuda.current_stream().wait_stream(s)
        # with a process group up, its watchdog thread queries work events while we capture:
        # thread-local capture mode keeps those queries legal (capture.graph)
        mode = "thread_local" if (dist.is_available() and dist.is_initialized()) else "global"
        for k in (0, 1):
            g = torch.cuda.CUDAGraph()
            with capture.graph(g, capture_error_mode=mode):
                self.outs[k] = self._body(k)
            self.graphs[k] = g
        torch.cuda.synchronize()
        for t, v in zip(self._state(), saved):
            t.copy_(v)
        tr.opt.step_count = step_count
        torch.cuda.synchronize()
        self.k = 0
        self.loaded = True
        self.first = True
        self.pending = None

    def _announced(self, src, dst) -> bool:
        """(src, dst) are the next_batch the previous step copied into the current set"""
        if self.pending is None:
            return False
        rs, rd, vs, vd, ps, pd, shape = self.pending
        return (rs() is src and rd() is dst and src._version == vs and dst._version == vd
                and (src.data_ptr(), dst.data_ptr(), tuple(src.shape)) == (ps, pd, shape))

    def _load(self, k, src, dst, gt_R, gt_t):
        self.src[k].copy_(src)
        self.dst[k].copy_(dst)
        self.gR[k].copy_(gt_R)
        self.gt[k].copy_(gt_t)

    def step(self, src, dst, gt_R, gt_t, next_batch=None):
        """One training step on (src, dst, gt_R, gt_t), and the level-1 selections of
        ``next_batch`` (default: the same batch again) on the side stream.  When (src, dst) are
        the tensors the previous step was given as ``next_batch``, unchanged since (the same
        objects, version counters and storage), the replay uses the set and selections that
        step prepared; any other batch is copied in and its selections computed first, so a
        step always trains on the points it is given.  -> (loss, l_R, l_t), static tensors
        overwritten by the next replay."""
        if not self.loaded:
            raise RuntimeError("GraphTrainer.capture() first")
        k = self.k
        nb = next_batch if next_batch is not None else (src, dst)
        if self.first or not self._announced(src, dst):  # nothing prefetched for this batch
            self.src[k].copy_(src)
            self.dst[k].copy_(dst)
            self._sel_into(k)
            self.first = False
        self.pending = Level1Prefetch._key(nb[0], nb[1])
        # the set this replay consumes holds (src, dst) since the previous replay's prefetch
        self.gR[k].copy_(gt_R)
        self.gt[k].copy_(gt_t)
        self.src[1 - k].copy_(nb[0])
        self.dst[1 - k].copy_(nb[1])
        self._set_scalars()
        self.graphs[k].replay()
        self.tr.opt.step_count += 1
        self.k = 1 - k
        return self.outs[k]
