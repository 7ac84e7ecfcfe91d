#!/bin/bash
# r5p: merge factor sweeps at the default 48 steps -- HRegNet 2 / 3 / 4, Model_V2 8 / 12 / 24.
set -o pipefail
O=gpurun_out/r5p; mkdir -p $O
run() {  # TAG ARGS
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-latency --no-eager-roofline $2 > $O/$1.json 2> $O/$1.err || { tail $O/$1.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$1.json')); print('$1', d['value'], d['ms_per_step'], d['config'].get('merge'), d['config']['executor'][:60])"
}
for r in 1 2; do
  for m in 2 3 4; do run h48m$m.$r "--merge $m"; done
  for m in 8 12 24; do run v48m$m.$r "--model v2 --merge $m"; done
done
