#!/bin/bash
# V2 executor sweep (r6): lanes x merge x front streaming, at --steps 48
set -o pipefail
O=gpurun_out/r6v2; mkdir -p $O
for cfg in "--lanes 2 --merge 12" "--lanes 2 --merge 24" "--lanes 4 --merge 12" "--lanes 4 --merge 6" "--lanes 2 --merge 8" "--lanes 8 --merge 6"; do
  for sw in "" "V2_FRONT_STREAM=1" "L1_LDS_MAX_N=65536"; do
    t=$(echo "$cfg $sw" | tr -c 'a-zA-Z0-9' _)
    HREG_SWITCHES=$sw timeout -k 10 200 python bench.py --model v2 --steps 48 --warmup 12 --no-cpu-baseline --no-latency $cfg > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -3 $O/$t.err; continue; }
    python -c "import json; d=json.load(open('$O/$t.json')); print('$cfg', '$sw', d['value'], d['ms_per_step'])"
  done
done
