#!/bin/bash
# Executor probes (configs[1], one box): reference batches merged per forward (--merge) at the
# driver's --steps 20 --warmup 5 and at 48 steps; host submit time vs elapsed.
set -o pipefail
O=gpurun_out/r5m; mkdir -p $O
run() {  # TAG ARGS
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-latency --no-eager-roofline $2 > $O/$1.json 2> $O/$1.err || { tail $O/$1.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$1.json')); print('$1', d['value'], d['ms_per_step'], 'host_submit_ms', d['host_submit_ms'], 'elapsed_ms', round(d['ms_per_step']*d['steps'],3))"
}
for r in 1 2; do
for m in 1 2 4 5 10 20; do run s20m$m.$r "--steps 20 --warmup 5 --merge $m"; done
done
for m in 4 6 8; do run s48m$m "--steps 48 --merge $m"; done
