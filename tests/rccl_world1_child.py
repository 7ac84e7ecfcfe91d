"""Child process of tests/test_gpu_train_ddp.py::test_graph_trainer_rccl_world1: a 1-rank
nccl (RCCL) process group, the captured training step with the bucket all-reduce as a graph
node, against the eager world-1 trainer.  Prints RESULT {json} lines; the teardown order is
graphs -> trainers -> synchronize -> destroy_process_group."""
import gc
import json
import os
import socket
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def report(**kw):
    print("RESULT " + json.dumps(kw), flush=True)


def main():
    from test_gpu_train_capture import _batches, _trainer
    from pcd_reg_hregnet_amd import _lib, trainer
    _lib.load()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ["MASTER_PORT"] = str(s.getsockname()[1])
    s.close()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    calls = []
    orig = dist.all_reduce

    def counting(t, *a, **k):
        calls.append(t.numel())
        return orig(t, *a, **k)
    B, n = 2, 4096
    batches = _batches(B, n, 4)
    plain = _trainer()
    red = _trainer()
    red.always_reduce = True
    dist.all_reduce = counting
    try:
        le = [plain.step(*batches[0])[0].clone()]
        lr_ = [red.step(*batches[0])[0].clone()]
        torch.cuda.synchronize()
        report(eager_calls=len(calls), eager_equal=bool(torch.equal(le[0], lr_[0]) and
                                                        torch.equal(plain.params.flat, red.params.flat)))
        calls.clear()
        gt = trainer.GraphTrainer(red, B, n)
        gt.capture(*batches[1])
        n_capture = len(calls)
        report(capture_calls=n_capture)
        for i in range(1, 4):
            nxt = batches[i + 1][:2] if i + 1 < 4 else None
            le.append(plain.step(*batches[i], next_batch=nxt)[0].clone())
            lr_.append(gt.step(*batches[i], next_batch=nxt)[0].clone())
        torch.cuda.synchronize()
        report(replay_calls=len(calls) - n_capture)
    finally:
        dist.all_reduce = orig
    report(losses=[float(x) for x in le], losses_rccl_graph=[float(x) for x in lr_],
           losses_equal=all(bool(torch.equal(a, b)) for a, b in zip(le, lr_)),
           params_equal=bool(torch.equal(plain.params.flat, red.params.flat)),
           moments_equal=bool(torch.equal(plain.opt.m, red.opt.m) and torch.equal(plain.opt.v, red.opt.v)),
           buffers_equal=all(bool(torch.equal(a, b)) for (_, a), (_, b) in
                             zip(plain.net.named_buffers(), red.net.named_buffers())))
    # teardown: the graphs holding the communicator's kernels first, then the communicator
    del gt
    del red, plain
    gc.collect()
    torch.cuda.synchronize()
    dist.destroy_process_group()
    report(teardown="ok")


if __name__ == "__main__":
    main()
