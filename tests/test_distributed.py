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


def test_single_process_path_has_no_collective():
    import bench
    assert bench.max_over_ranks(1.25, torch.device("cpu")) == 1.25
    s0 = bench.shard_batch(0, 1, 1024)[0]
    s1 = bench.shard_batch(1, 1, 1024)[0]
    assert not np.array_equal(s0, s1)
