#!/bin/bash
# stage-1 split, index vs kNN, Morton (new) and cell-ordered (old) index (gpurun_out/s1s2/)
set -o pipefail
O=gpurun_out/s1s2; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for lib in new old; do
    L=""; [ $lib = old ] && L=$PWD/pcd_reg_hregnet_amd/ab_simold.so
    for v in 0 3 2; do
      t=$lib.skip$v.$r
      HREG_LIB=$L HREG_SWITCHES=PROBE_S1_SKIP=$v timeout -k 10 300 python bench.py --allow-probes --steps 48 --warmup 5 --no-cpu-baseline > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail $O/$t.err; exit 1; }
      python -c "import json; d=json.load(open('$O/$t.json')); print('$t', d['value'], d['ms_per_step'])"
    done
  done
done
