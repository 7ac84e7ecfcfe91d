"""Per-launch times of the train-mode BN kernels (hreg_bn_stats: col_reduce<0> + finalize;
hreg_bn_backward: col_reduce<1> + finalize + bn_backward; hreg_bn_apply) at level-1 sizes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pcd_reg_hregnet_amd import _lib, train  # noqa: E402


def t_us(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


st = torch.cuda.current_stream().cuda_stream
for R, C in ((524288, 32), (524288, 64), (262144, 128)):
    y = torch.randn(R, C, device="cuda")
    dout = torch.randn(R, C, device="cuda")
    mean, invstd, var = (torch.empty(C, device="cuda") for _ in range(3))
    g, b = torch.rand(C, device="cuda"), torch.randn(C, device="cuda")
    ws = train.col_reduce_ws(R, C, y.device)
    dy, dg, db = torch.empty_like(y), torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    out = torch.empty_like(y)
    s = t_us(lambda: _lib.call("hreg_bn_stats", y, R, C, 1e-5, ws, mean, invstd, var, st))
    ap = t_us(lambda: _lib.call("hreg_bn_apply", y, R, C, mean, invstd, g, b, 1, out, st))
    bw = t_us(lambda: _lib.call("hreg_bn_backward", dout, None, y, R, C, mean, invstd, g, b, 1, ws, dy, dg, db, 0, st))
    bwo = t_us(lambda: _lib.call("hreg_bn_backward", dout, out, y, R, C, mean, invstd, g, b, 1, ws, dy, dg, db, 0, st))
    mb = R * C * 4 / 1e6
    print(f"R={R} C={C} ({mb:.0f} MB/stream): stats {s:.1f} us, apply {ap:.1f}, backward {bw:.1f} "
          f"(with out {bwo:.1f})", flush=True)
