"""Eager Trainer vs GraphTrainer, step by step (losses and the first step whose parameters
differ): usage python tools/graph_train_check.py [B] [N] [steps] [same|vary]"""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_train_capture import _trainer, _batches  # noqa: E402


def main():
    from pcd_reg_hregnet_amd import _lib, trainer
    _lib.load()
    B, N, steps = (int(a) for a in sys.argv[1:4])
    same = sys.argv[4] == "same"
    batches = _batches(B, N, 1 if same else steps + 1)
    get = (lambda i: batches[0]) if same else (lambda i: batches[i])
    eager, graphed = _trainer(), _trainer()
    gt = trainer.GraphTrainer(graphed, B, N)
    gt.capture(*get(0))
    for i in range(steps):
        nxt = get(i + 1)[:2]
        le = float(eager.step(*get(i), next_batch=nxt)[0])
        lg = float(gt.step(*get(i), next_batch=nxt)[0])
        same_p = torch.equal(eager.params.flat, graphed.params.flat)
        print(f"step {i}: eager {le:.7f} graph {lg:.7f} params equal {same_p}", flush=True)


if __name__ == "__main__":
    main()
