#!/bin/bash
# stage-1 cost with the Morton (new) and cell-ordered (old, ab_simold.so) spatial index: bench lines
# with and without the streamed stage 1 (PROBE_NO_S1), 48 steps (outputs gpurun_out/sip/).
set -o pipefail
O=gpurun_out/sip; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in new old; do
    L=""; [ $v = old ] && L=$PWD/pcd_reg_hregnet_amd/ab_simold.so
    for s in 0 1; do
      HREG_LIB=$L HREG_SWITCHES=PROBE_NO_S1=$s timeout -k 10 300 python bench.py --steps 48 --warmup 5 --no-cpu-baseline > $O/$v.$s.$r.json 2> $O/$v.$s.$r.err || { echo "$v failed"; tail $O/$v.$s.$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/$v.$s.$r.json')); print('$v nos1=$s', d['value'], d['ms_per_step'])"
    done
  done
done
