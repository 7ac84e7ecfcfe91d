#!/bin/bash
# stage-1 cost split: bench lines with the whole stage 1, without its FPS, without its kNN, without
# it, 20 and 48 steps (gpurun_out/s1s/)
set -o pipefail
O=gpurun_out/s1s; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in PROBE_S1_SKIP=0 PROBE_S1_SKIP=1 PROBE_S1_SKIP=2 PROBE_NO_S1=1; do
    for st in 20 48; do
      t=$(echo $v | tr '=' '_').s$st.$r
      HREG_SWITCHES=$v timeout -k 10 300 python bench.py --allow-probes --steps $st --warmup 5 --no-cpu-baseline > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail $O/$t.err; exit 1; }
      python -c "import json; d=json.load(open('$O/$t.json')); print('$t', d['value'], d['ms_per_step'])"
    done
  done
done
