#!/bin/bash
# r5r: the descriptor-space kNN with 4 queries per wave (HREG_KNND_QW): kNN tests, the op alone
# against one query per wave, paired bench lines; then a kernel trace of the training step.
set -o pipefail
O=gpurun_out/r5r; mkdir -p $O
export TMPDIR=/tmp
HREG_LIB=$PWD/pcd_reg_hregnet_amd/ab_qw4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -m gpu -q -rf --timeout 300 \
  --timeout-method thread -k "knn or vs_oracle_lidar or reference_fixture" > $O/pytest.log 2>&1 \
  || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
HREG_LIB=$PWD/pcd_reg_hregnet_amd/ab_qw4.so timeout -k 10 120 python tools/op_bench.py knn --b 64 > $O/op_qw4.txt 2>&1 || { tail $O/op_qw4.txt; exit 1; }
timeout -k 10 120 python tools/op_bench.py knn --b 64 > $O/op_qw1.txt 2>&1 || { tail $O/op_qw1.txt; exit 1; }
grep -h knn_desc $O/op_qw4.txt $O/op_qw1.txt
bash tools/ab_lines.sh r5r_ab 2 "--steps 20 --warmup 5 --no-latency --no-eager-roofline" - lib:ab_qw4.so || exit 1
bash tools/train_trace.sh r5t
