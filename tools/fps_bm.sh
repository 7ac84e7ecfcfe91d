#!/bin/bash
# FPS winner-slot mask from the lane's own max (HREG_FPS_BESTMASK, default) vs from the wave max
# (ab_bm0.so): FPS exactness tests, then bench lines with the fps entry (gpurun_out/fbm/)
set -o pipefail
O=gpurun_out/fbm; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -q -rf --timeout 300 --timeout-method thread -k "fps" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in new bm0; do
    L=""; [ $v = bm0 ] && L=$PWD/pcd_reg_hregnet_amd/ab_bm0.so
    for st in 20 48; do
      HREG_LIB=$L timeout -k 10 300 python bench.py --steps $st --warmup 5 --no-cpu-baseline > $O/$v.s$st.$r.json 2> $O/$v.s$st.$r.err || { echo "$v failed"; tail $O/$v.s$st.$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/$v.s$st.$r.json')); f=d['fps']; print('$v s$st', d['value'], d['ms_per_step'], f['us_per_iteration'], f['frac_floor_over_kernel'])"
    done
  done
done
