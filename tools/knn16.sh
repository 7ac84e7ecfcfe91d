#!/bin/bash
# 16-point-block indexed kNN: index / kNN exactness tests, op micro-bench, bench lines against the
# 12-bit-cell index (ab_simold.so) at 20 and 48 steps (gpurun_out/k16/)
set -o pipefail
O=gpurun_out/k16; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -q -rf --timeout 300 --timeout-method thread -k "spatial or knn or lidar or graph" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
echo "new $(timeout -k 10 200 python tools/op_bench.py knn)"
echo "old $(HREG_LIB=$PWD/pcd_reg_hregnet_amd/ab_simold.so timeout -k 10 200 python tools/op_bench.py knn)"
for r in 1 2; do
  for v in new old; do
    L=""; [ $v = old ] && L=$PWD/pcd_reg_hregnet_amd/ab_simold.so
    for st in 20 48; do
      HREG_LIB=$L timeout -k 10 300 python bench.py --steps $st --warmup 5 --no-cpu-baseline > $O/$v.s$st.$r.json 2> $O/$v.s$st.$r.err || { echo "$v failed"; tail $O/$v.s$st.$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/$v.s$st.$r.json')); print('$v s$st', d['value'], d['ms_per_step'])"
    done
  done
done
