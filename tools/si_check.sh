#!/bin/bash
# Morton index (radix) + multi-block kNN variants: order / kNN exactness tests, op micro-bench and
# bench lines: new (Morton, 1 block per trip), m2 / m4 (Morton, 2 / 4 blocks per trip), old
# (12-bit cell index) (gpurun_out/sic/)
set -o pipefail
O=gpurun_out/sic; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -q -rf --timeout 300 --timeout-method thread -k "spatial or knn" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
lib() { case $1 in new) echo "";; old) echo $PWD/pcd_reg_hregnet_amd/ab_simold.so;; *) echo $PWD/pcd_reg_hregnet_amd/ab_$1.so;; esac; }
for v in new m2 m4 old; do
  echo "$v $(HREG_LIB=$(lib $v) timeout -k 10 200 python tools/op_bench.py knn)"
done
for r in 1 2; do
  for v in new m2 m4 old; do
    for st in 20 48; do
      [ $st = 48 ] && [ $r = 2 ] && continue
      HREG_LIB=$(lib $v) timeout -k 10 300 python bench.py --steps $st --warmup 5 --no-cpu-baseline > $O/$v.s$st.$r.json 2> $O/$v.s$st.$r.err || { echo "$v failed"; tail $O/$v.s$st.$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/$v.s$st.$r.json')); print('$v s$st', d['value'], d['ms_per_step'])"
    done
  done
done
