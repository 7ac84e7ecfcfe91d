"""Single-batch latency under a kernel trace: the 1-lane GraphPipeline (bench.py's `latency`
graph figure) replayed alone, with idle gaps between replays so tools/timeline.py can split them.

  rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/latency_trace.py [B]
  python tools/timeline.py OUT/.../run_kernel_trace.csv group_l1_6_kernel --list
"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from pcd_reg_hregnet_amd import _lib, engine  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    _lib.load()
    device = torch.device("cuda", 0)
    P = bench.make_model(device).prepared(device)
    s, d, _, _ = bench.shard_batch(0, B, 16384)
    src, dst = torch.from_numpy(s).to(device), torch.from_numpy(d).to(device)
    with torch.no_grad():
        gp = engine.GraphPipeline(P, src, dst, lanes=1)
        ts = []
        for i in range(8):
            torch.cuda.synchronize()
            time.sleep(0.005)
            t0 = time.perf_counter()
            gp.run_forwards(1)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
    print("replay ms:", " ".join(f"{t:.3f}" for t in ts), flush=True)


if __name__ == "__main__":
    main()
