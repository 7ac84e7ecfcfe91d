#!/bin/bash
# r5s: CoarseReg's 512-channel head on two row tiles (HREG_CORR512_JT=2 build): its bitwise test
# in both builds, then paired bench lines (+ the descriptor kNN at 8 queries per wave).
set -o pipefail
O=gpurun_out/r5s; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -m gpu -q -rf --timeout 200 --timeout-method thread \
  -k "coarse_head_row_tiles" > $O/pytest_base.log 2>&1 || { echo "base test failed"; tail -30 $O/pytest_base.log; exit 1; }
tail -1 $O/pytest_base.log
HREG_LIB=$PWD/pcd_reg_hregnet_amd/ab_c512jt2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -m gpu -q -rf \
  --timeout 200 --timeout-method thread -k "coarse_head_row_tiles or vs_oracle_lidar" > $O/pytest_jt2.log 2>&1 \
  || { echo "jt2 test failed"; tail -30 $O/pytest_jt2.log; exit 1; }
tail -1 $O/pytest_jt2.log
HREG_LIB=$PWD/pcd_reg_hregnet_amd/ab_qw8.so timeout -k 10 120 python tools/op_bench.py knn --b 64 > $O/op_qw8.txt 2>&1 || { tail $O/op_qw8.txt; exit 1; }
grep -h knn_desc $O/op_qw8.txt
bash tools/ab_lines.sh r5s_ab 2 "--steps 20 --warmup 5 --no-latency" - lib:ab_c512jt2.so lib:ab_qw8.so
