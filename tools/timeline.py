"""Timeline of a rocprofv3 --kernel-trace run of bench.py (graph executor).

  python tools/timeline.py <kernel_trace.csv> [marker_kernel]

Splits the trace into segments separated by idle gaps > 0.3 ms (the host synchronises
between the warm-up, the timed region and the instrumented eager pass), and for every segment
prints its length, how many forwards it ran (launches of the marker kernel, default the level-1
kernel) and, for the segments that ran forwards, the busy / idle split and a profile of how many
kernels ran at once: the time with exactly one kernel in flight is where a round's head or tail
leaves the GPU to one lane's serial chain.  The kernels active during the single-kernel time
are listed.
"""
import csv
import sys
from collections import defaultdict


def load(path):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:70]


def segments(rows, gap_ns=300_000):
    segs, cur, end = [], [], None
    for s, e, n in rows:
        if cur and s - end > gap_ns:
            segs.append(cur)
            cur, end = [], None
        cur.append((s, e, n))
        end = e if end is None else max(end, e)
    if cur:
        segs.append(cur)
    return segs


def profile(seg):
    ev = []
    for s, e, n in seg:
        ev.append((s, 1, n))
        ev.append((e, -1, n))
    ev.sort(key=lambda x: (x[0], x[1]))
    t0 = ev[0][0]
    conc = defaultdict(int)
    alone = defaultdict(int)
    active = defaultdict(int)
    k, last = 0, t0
    for t, d, n in ev:
        if t > last:
            conc[min(k, 8)] += t - last
            if k == 1:
                (only,) = [m for m, c in active.items() if c > 0]
                alone[only] += t - last
        k += d
        active[n] += d
        last = t
    return conc, alone


def listing(seg):
    """every kernel of a segment in start order: offset, duration, idle time before it (no kernel
    in flight) and the kernels in flight when it starts"""
    t0 = seg[0][0]
    end = t0
    for s, e, n in seg:
        live = sum(1 for s2, e2, _ in seg if s2 < s and e2 > s)
        idle = max(0, s - end)
        print(f"   {(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  idle {idle / 1e3:6.1f}  "
              f"with {live}  {short(n)}")
        end = max(end, e)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    rows = load(args[0])
    marker = args[1] if len(args) > 1 else "group_l1_6_kernel"
    segs = segments(rows)
    last1 = None
    for i, seg in enumerate(segs):
        span = max(e for _, e, _ in seg) - seg[0][0]
        fw = sum(1 for _, _, n in seg if marker in n)
        print(f"segment {i}: {span / 1e6:.3f} ms, {len(seg)} kernels, {fw} x {marker}")
        if fw == 1:
            last1 = seg
        if fw < 2:
            continue
        conc, alone = profile(seg)
        tot = sum(conc.values())
        print("   in flight: " + ", ".join(f"{k}{'+' if k == 8 else ''}: {v / 1e6:.3f} ms ({100 * v / tot:.1f} %)"
                                         for k, v in sorted(conc.items())))
        print(f"   per forward: {span / fw / 1e6:.4f} ms")
        for n, v in sorted(alone.items(), key=lambda kv: -kv[1])[:8]:
            print(f"     alone {v / 1e6:.3f} ms  {short(n)}")
    if "--list" in sys.argv and last1:
        # the last one-forward segment (the latency run's last replay)
        print("last single-forward segment:")
        listing(last1)


if __name__ == "__main__":
    main()
