#!/bin/bash
# What the streamed stage 1 (level-1 FPS + spatial index + kNN of the next round) costs a round:
# bench lines with and without it (PROBE_NO_S1; static inputs keep the buffers valid), 20 and 48
# steps (outputs gpurun_out/s1p/).
set -o pipefail
O=gpurun_out/s1p; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in PROBE_NO_S1=0 PROBE_NO_S1=1; do
    for st in 20 48; do
      t=$(echo $v | tr '=' '_').s$st.$r
      HREG_SWITCHES=$v timeout -k 10 300 python bench.py --steps $st --warmup 5 --no-cpu-baseline > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail $O/$t.err; exit 1; }
      python -c "import json; d=json.load(open('$O/$t.json')); print('$t', d['value'], d['ms_per_step'], round(d['ms_per_step'] * $st, 2))"
    done
  done
done
