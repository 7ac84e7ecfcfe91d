"""roofline.in_executor's source: the level kernels' durations inside the
timed graph executor, from a rocprofv3 kernel trace of

    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- \
        python3 bench.py --steps S --warmup W --no-eager-roofline --no-latency --no-cpu-baseline

With --no-eager-roofline the timed region's replays are the run's last dispatches of every
level kernel (the FPS diagnostics after it launch no level kernel), so the mean over the last
S dispatches of each is its in-executor launch duration; union_us is the time at least one of
those launches was running (the level kernels of different lanes overlap each other and the
rest of the round).

    python tools/in_executor.py DIR KEY S OUT.json [TREE]
    (KEY = hregnet:b8:n16384:s20; OUT.json is updated in place, one entry per KEY)
"""
import csv
import glob
import json
import os
import sys

LEVEL_KERNELS = ("group_l1_6_kernel", "group_fused6_kernel", "group_split6j_kernel")


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("<")[0].strip()


def main():
    d, key, steps, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    tree = sys.argv[5] if len(sys.argv) > 5 else None
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {d}")
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    per = {}
    iv = []
    for k in LEVEL_KERNELS:
        ds = [(e - s) / 1e3 for s, e, n in rows if n == k]
        if not ds:  # (one level-3 form runs: split6j or split6p)
            continue
        if len(ds) < steps:
            raise SystemExit(f"{k}: {len(ds)} dispatches < {steps}")
        last = ds[-steps:]
        per[k] = round(sum(last) / len(last), 2)
        iv += [(s_, e) for s_, e, n in rows if n == k][-steps:]
    # the time at least one level kernel of the timed replays was running (overlaps counted once)
    iv.sort()
    union, (cs, ce) = 0, iv[0]
    for s_, e in iv[1:]:
        if s_ > ce:
            union, cs, ce = union + ce - cs, s_, e
        else:
            ce = max(ce, e)
    union += ce - cs
    try:
        doc = json.load(open(out))
    except (OSError, ValueError):
        doc = {}
    doc[key] = {"avg_us": per, "dispatches": steps, "tree": tree, "union_us": round(union / 1e3, 2),
                "basis": "mean duration of the last S dispatches of each level kernel in a "
                         "rocprofv3 --kernel-trace run of bench.py --no-eager-roofline (the timed "
                         "graph replays)"}
    json.dump(doc, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(doc[key]))


if __name__ == "__main__":
    main()
