"""The N>1 bench path on CPU: world_size-2 gloo ranks shard disjoint pairs, run no
collective on the data path, and reduce only the elapsed time (max over ranks)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    s, d, R, t = bench.shard_batch(rank, 2, 2048)
    el = bench.max_over_ranks(0.5 + rank, torch.device("cpu"))
    v = bench.job_throughput(2, 10, world, el)
    # checksum of this rank's shard to show shards are disjoint
    q.put((rank, float(s.sum()), float(d.sum()), el, v))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_bench_path(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    sums = {(r[1], r[2]) for r in res}
    assert len(sums) == world                        # disjoint shards
    assert all(r[3] == 0.5 + world - 1 for r in res)  # max over ranks
    assert all(abs(r[4] - 2 * 10 * world / (0.5 + world - 1)) < 1e-9 for r in res)


@pytest.mark.parametrize("world", [2, 3])
def test_bench_launcher_starts_n_ranks(world):
    """`python bench.py --gpus N` with no torchrun: the script starts
    N rank processes itself, each initialises the process group with world size N, shards
    its own pairs, and the elapsed time is the max over ranks."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(world),
                        "--launch-check", "--backend", "gloo"], env=env, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == list(range(world))
    assert all(x["world"] == world for x in lines)
    assert len({x["shard_sum"] for x in lines}) == world         # disjoint shards
    assert all(x["elapsed_max"] == 0.5 + world - 1 for x in lines)
    assert all(abs(x["value"] - 10 * world / (0.5 + world - 1)) < 1e-9 for x in lines)


def test_bench_rejects_world_mismatch():
    """A rank whose WORLD_SIZE differs from --gpus exits non-zero instead of reporting."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--launch-check", "--backend", "gloo"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE=1" in p.stderr


def test_single_process_path_has_no_collective():
    import bench
    assert bench.max_over_ranks(1.25, torch.device("cpu")) == 1.25
    s0 = bench.shard_batch(0, 1, 1024)[0]
    s1 = bench.shard_batch(1, 1, 1024)[0]
    assert not np.array_equal(s0, s1)


def _bucket_worker(rank, world, port, q):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pcd_reg_hregnet_amd.train import GradBucket
    torch.manual_seed(0)
    params = [torch.nn.Parameter(torch.randn(5, 3)), torch.nn.Parameter(torch.randn(7)),
              torch.nn.Parameter(torch.randn(2, 2), requires_grad=False)]
    b = GradBucket(params)
    b.attach()
    # rank-dependent "backward": one grad written in place, one allocated separately
    params[0].grad.add_(float(rank + 1))
    params[1].grad = torch.full((7,), 10.0 * (rank + 1))
    b.collect()
    # the trainer's collective (trainer.ddp_average, eager and captured steps alike): exactly
    # one all_reduce per step, over the whole flat bucket (every gradient in parameter order)
    from pcd_reg_hregnet_amd import trainer as T
    calls = []
    orig = dist.all_reduce

    def counting(t, *a, **k):
        calls.append((t.data_ptr(), t.numel()))
        return orig(t, *a, **k)
    dist.all_reduce = counting
    try:
        T.ddp_average(b)
    finally:
        dist.all_reduce = orig
    one_collective = calls == [(b.flat.data_ptr(), b.flat.numel())]
    # the trainer's flat parameters: rank 0's values everywhere after the broadcast
    from pcd_reg_hregnet_amd.trainer import FlatParams
    mine = [torch.nn.Parameter(torch.full((5, 3), float(rank))),
            torch.nn.Parameter(torch.full((7,), 3.0 + rank))]
    fp = FlatParams(mine)
    fp.broadcast(0)
    synced = (torch.equal(mine[0].detach(), torch.zeros(5, 3)) and
              torch.equal(mine[1].detach(), torch.full((7,), 3.0)) and
              mine[1].data_ptr() == fp.flat.data_ptr() + 64 * 4)
    # numpy copies: a tensor on a multiprocessing queue travels as a shared-memory fd
    # that the receiver can only open while this process is still alive
    q.put((rank, params[0].grad.numpy().copy(), params[1].grad.numpy().copy(), b.flat.numel(),
           params[0].grad.data_ptr() == b.flat.data_ptr() and
           params[1].grad.data_ptr() == b.flat.data_ptr() + 64 * 4, synced, one_collective))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_grad_bucket_all_reduce():
    """The training step's gradient bucket (config 4): all trainable
    gradients in one flat buffer, one all_reduce, averaged; .grad are views into it."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=120) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for _, g0, g1, n, view, synced, one_collective in res:
        assert n == 128 and view  # 5x3 + 7 trainable floats, each padded to 64 (256 B)
        assert synced and one_collective
        assert torch.equal(torch.from_numpy(g0), torch.full((5, 3), 1.5))   # mean of 1 and 2
        assert torch.equal(torch.from_numpy(g1), torch.full((7,), 15.0))    # mean of 10 and 20


def _trainer_step_worker(rank, world, port, q):
    """A real trainer.Trainer.step on gloo: the rank's gradients come from a stub
    local_gradients (the train-mode forward needs the GPU), Adam from a stub that records the
    bucket it sees; everything else -- prefetch lookup, ddp_average, the bucket's all_reduce,
    the division -- is the trainer's own code.  dist.all_reduce is wrapped to count calls."""
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pcd_reg_hregnet_amd import trainer as T
    torch.manual_seed(rank)  # different initial values: the broadcast must win
    net = torch.nn.Sequential(torch.nn.Linear(3, 5), torch.nn.Linear(5, 2))
    tr = T.Trainer(net, lr=1e-3)
    log = []

    def local_gradients(src, dst, gt_R, gt_t, hook=None):
        tr.bucket.attach()
        try:
            for i, p in enumerate(tr.params.params):
                p.grad.add_(float((rank + 1) * (i + 1)))
            tr.bucket.collect()
        finally:
            T.GradBucket.direct_off()
        log.append("local")
        z = torch.zeros(())
        return z, z, z
    tr.local_gradients = local_gradients
    seen = []
    tr.opt.step = lambda: (log.append("adam"), seen.append(tr.bucket.flat.clone()))
    calls = []
    orig = dist.all_reduce

    def counting(t, *a, **k):
        calls.append((t.data_ptr(), t.numel()))
        log.append("all_reduce")
        return orig(t, *a, **k)
    dist.all_reduce = counting
    try:
        x = torch.zeros(1, 4, 3)
        for _ in range(3):
            tr.step(x, x, torch.eye(3)[None], torch.zeros(1, 3))
    finally:
        dist.all_reduce = orig
    flat = tr.params.flat.clone()
    q.put((rank, calls == [(tr.bucket.flat.data_ptr(), tr.bucket.flat.numel())] * 3,
           log == ["local", "all_reduce", "adam"] * 3,
           [g.numpy().copy() for g in seen], flat.numpy().copy(),
           [p.numel() for p in tr.params.params]))
    dist.barrier()
    dist.destroy_process_group()


def test_trainer_step_issues_one_collective():
    """a real Trainer.step on two gloo ranks issues exactly one
    all_reduce per step, over the whole flat gradient bucket, after the rank's backward and
    before Adam; Adam sees the mean of the ranks' gradients; both ranks start from rank 0's
    parameters (replaces the source-text count of r4)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_trainer_step_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=120) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    from pcd_reg_hregnet_amd.train import flat_offsets
    for rank, one_per_step, order, seen, flat, sizes in res:
        assert one_per_step and order, rank
        offs, n = flat_offsets([torch.empty(k) for k in sizes])
        for g in seen:
            for i, (o, k) in enumerate(zip(offs, sizes)):
                # mean over ranks of (rank + 1) * (i + 1): 1.5 * (i + 1)
                assert np.array_equal(g[o:o + k], np.full(k, 1.5 * (i + 1), np.float32))
    assert np.array_equal(res[0][4], res[1][4])  # broadcast: the same parameters


def test_train_bodies_share_ddp_average():
    """The captured GraphTrainer body reduces through the same call as Trainer.step
    (trainer.ddp_average, after the bucket collect, before Adam); its execution on RCCL is
    tests/test_gpu_train_ddp.py::test_graph_trainer_rccl_world1."""
    import inspect
    from pcd_reg_hregnet_amd import trainer as T
    body = inspect.getsource(T.GraphTrainer._body)
    assert body.index("collect(") < body.index("ddp_average(") < body.index("hreg_adam_step_dev")
