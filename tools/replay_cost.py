"""Host cost of a graph replay vs its GPU time (GraphPipeline, configs[1] batch): for each lane
count, the wall time of the replay() call itself (host submission), and of replay + synchronize.
usage: python tools/replay_cost.py [lanes ...]"""
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from pcd_reg_hregnet_amd import engine  # noqa: E402


def main():
    dev = torch.device("cuda")
    net = bench.make_model(dev)
    P = net.prepared(dev)
    s, d, _, _ = bench.shard_batch(0, bench.PAIRS_PER_GPU, bench.POINTS)
    src, dst = torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev)
    for lanes in [int(x) for x in sys.argv[1:]] or [20, 48]:
        with torch.no_grad():
            gp = engine.GraphPipeline(P, src, dst, lanes=lanes)
            gp.run_forwards(lanes, stream=True)
            torch.cuda.synchronize()
            for rep in range(3):
                g = gp.g_step[gp.ready]
                t0 = time.perf_counter()
                g.replay()
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                gp.ready = 1 - gp.ready
                time.sleep(0.005)  # (an idle gap: tools/timeline.py splits the trace here)
                print(f"lanes {lanes}: replay() call {1e3 * (t1 - t0):.3f} ms, replay + sync "
                      f"{1e3 * (t2 - t0):.3f} ms = {1e3 * (t2 - t0) / lanes:.4f} ms/forward", flush=True)
        del gp
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
