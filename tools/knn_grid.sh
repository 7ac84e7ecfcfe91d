#!/bin/bash
# capped indexed-kNN grid (HREG_KNN_GRID variants ab_g*.so): exactness tests on one variant, then
# bench lines at 20 and 48 steps against the default grid (gpurun_out/kg/)
set -o pipefail
O=gpurun_out/kg; mkdir -p $O
export TMPDIR=/tmp
HREG_LIB=$PWD/pcd_reg_hregnet_amd/ab_g512.so timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -q -rf --timeout 300 --timeout-method thread -k "indexed" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in base g256 g512 g1024; do
    L=""; [ $v != base ] && L=$PWD/pcd_reg_hregnet_amd/ab_$v.so
    for st in 20 48; do
      HREG_LIB=$L timeout -k 10 300 python bench.py --steps $st --warmup 5 --no-cpu-baseline > $O/$v.s$st.$r.json 2> $O/$v.s$st.$r.err || { echo "$v failed"; tail $O/$v.s$st.$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/$v.s$st.$r.json')); print('$v s$st', d['value'], d['ms_per_step'])"
    done
  done
done
