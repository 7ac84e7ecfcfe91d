"""Probe (HIP graph capture + autograd): a stream that joins a capture through another forked
stream's event ("nested fork") vs one that first joins from the origin stream and later waits on
the forked stream; noback: the same forward without autograd; leafcur: the leaf's first use on
the origin stream.  usage: python tools/micro/nested_fork_probe.py [nested|prejoined|noback|leafcur]"""
import sys

import torch


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "nested"
    x = torch.randn(4096, device="cuda", requires_grad=True)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def body():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        if mode == "prejoined":
            s2.wait_stream(cur)  # s2 joins from the origin first
        a0 = x * 2 if mode == "leafcur" else None
        s1.wait_stream(cur)
        with torch.cuda.stream(s1):
            a = a0 if a0 is not None else x * 2
            s2.wait_stream(s1)
            with torch.cuda.stream(s2):
                b = a * 3
            c = a * 4
            s1.wait_stream(s2)
            d = b * c
        cur.wait_stream(s1)
        loss = d.sum()
        if mode != "noback":
            x.grad = None
            loss.backward()
        cur.wait_stream(s1)
        cur.wait_stream(s2)
        return loss.detach()

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            body()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = body()
    g.replay()
    torch.cuda.synchronize()
    print(mode, "captured and replayed ok", float(out), flush=True)


if __name__ == "__main__":
    main()
