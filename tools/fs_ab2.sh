#!/bin/bash
# Front streaming A/B: plain rounds vs front streaming with each per-lane order (FRONT_ORDER),
# alternating, at --steps 20 --warmup 5 and 48 (outputs gpurun_out/fs2/).
set -o pipefail
O=gpurun_out/fs2; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in FRONT_STREAM=0 FRONT_ORDER=0 FRONT_ORDER=1 FRONT_ORDER=2; do
    for st in 20 48; do
      t=$(echo $v | tr '=' '_').s$st.$r
      HREG_SWITCHES=$v timeout -k 10 300 python bench.py --steps $st --warmup 5 --no-cpu-baseline > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail $O/$t.err; exit 1; }
      python -c "import json; d=json.load(open('$O/$t.json')); print('$t', d['value'], d['ms_per_step'])"
    done
  done
done
