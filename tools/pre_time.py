"""Eager timing of the chain kernels against the layerwise pair they replace (HIP events, the
median of 20 launches): hreg_ts_gemm_bn_pre vs hreg_bn_apply + hreg_ts_gemm_bn, and
hreg_gemm_tn_pre vs hreg_gemm_tn, at the training step's chain shapes.

usage: python tools/pre_time.py"""
import statistics

import torch


def timeit(fn, n=20):
    ts = []
    for _ in range(n + 3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(ts[3:])


def main():
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from pcd_reg_hregnet_amd import _lib, train
    lib = _lib.load()
    st = _lib.stream_handle()
    dev = torch.device("cuda")
    for R, K, N in [(131072, 64, 64), (131072, 64, 128), (524288, 32, 32), (524288, 32, 64), (32768, 128, 256),
                    (16384, 256, 256), (32768, 128, 128)]:
        g = torch.Generator(device=dev).manual_seed(0)
        y = torch.randn(R, K, device=dev, generator=g)
        W = torch.randn(N, K, device=dev, generator=g) * 0.1
        pm, pi = torch.randn(K, device=dev) * 0.1, torch.rand(K, device=dev) + 0.5
        pg, pb = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.1
        out = torch.empty(R, N, device=dev)
        act = torch.empty(R, K, device=dev)
        mean, invstd, var = (torch.empty(N, device=dev) for _ in range(3))
        ws = torch.empty(max(lib.hreg_ts_gemm_bn_ws_bytes(R, K, N), 16), dtype=torch.uint8, device=dev)

        def pre():
            _lib.call("hreg_ts_gemm_bn_pre", y, K, R, K, W, N, None, out, N, 1e-5, 0.1, ws, mean, invstd, var,
                      None, None, pm, pi, pg, pb, 1, st)

        def apply():
            _lib.call("hreg_bn_apply", y, R, K, pm, pi, pg, pb, 1, act, st)

        def plain():
            _lib.call("hreg_ts_gemm_bn", act, K, R, K, W, 0, N, None, out, N, 1e-5, 0.1, ws, mean, invstd, var,
                      None, None, st)
        dy = torch.randn(R, N, device=dev, generator=g)
        gws = torch.empty(max(lib.hreg_gemm_tn_ws_bytes(R, N, K), 16), dtype=torch.uint8, device=dev)
        dW = torch.empty(N, K, device=dev)

        def tn_pre():
            _lib.call("hreg_gemm_tn_pre", dy, N, y, K, R, N, K, 0.0, gws, dW, pm, pi, pg, pb, 1, st)

        def tn():
            _lib.call("hreg_gemm_tn", dy, N, act, K, R, N, K, 0.0, gws, dW, st)
        t = {k: round(timeit(f), 1) for k, f in (("ts_pre", pre), ("bn_apply", apply), ("ts_bn", plain),
                                                   ("tn_pre", tn_pre), ("tn", tn))}
        print(f"R {R} K {K} N {N}: {t}  fwd pre {t['ts_pre']} vs {t['bn_apply'] + t['ts_bn']:.1f}, "
              f"wgrad pre {t['tn_pre']} vs {t['tn']}", flush=True)


if __name__ == "__main__":
    main()
