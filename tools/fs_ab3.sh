#!/bin/bash
# Front streaming A/B (outputs gpurun_out/fs3/): plain rounds vs order 0 vs the two halves of a
# lane on two streams (order 3), at 20 steps and at 48 (front streaming forced on there).
set -o pipefail
O=gpurun_out/fs3; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in FRONT_STREAM=0 FRONT_ORDER=0 FRONT_ORDER=3; do
    for st in 20 48; do
      t=$(echo $v | tr '=' '_').s$st.$r
      HREG_SWITCHES=$v,FRONT_STREAM_MAX_LANES=48 timeout -k 10 300 python bench.py --steps $st --warmup 5 --no-cpu-baseline > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail $O/$t.err; exit 1; }
      python -c "import json; d=json.load(open('$O/$t.json')); print('$t', d['value'], d['ms_per_step'])"
    done
  done
done
