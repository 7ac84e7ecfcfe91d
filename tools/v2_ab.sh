#!/bin/bash
set -o pipefail
O=gpurun_out/v2ab; mkdir -p $O
timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline > $O/a.json 2> $O/a.err || { tail $O/a.err; exit 1; }
HREG_B6_L1=0 HREG_B6_L2=0 HREG_B6_L3=0 HREG_B6_HEADS=0 HREG_B6_MLP=0 HREG_FUSED_COARSE=0 HREG_B6_GEMM=0 timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline --executor pipeline > $O/c.json 2> $O/c.err || { tail $O/c.err; exit 1; }
python - <<'P'
import json
for f in "abc":
    d = json.load(open(f"gpurun_out/v2ab/{f}.json"))
    print(f, d["value"], d["ms_per_step"], {k: v["avg_launch_us"] for k, v in d["roofline"]["per_entry"].items()})
P
