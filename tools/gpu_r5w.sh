#!/bin/bash
# r5w: the xyz kNN kernels (knn3 / knn_group) with 4 queries per wave (HREG_KNN3_QW=4 build): the kNN
# and end-to-end tests on it, the ops alone, paired bench lines.
set -o pipefail
O=gpurun_out/r5w; mkdir -p $O
export TMPDIR=/tmp
HREG_LIB=$PWD/pcd_reg_hregnet_amd/ab_k3qw4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -m gpu -q -rf \
  --timeout 300 --timeout-method thread -k "knn or vs_oracle_lidar or reference_fixture or randsample" > $O/pytest.log 2>&1 \
  || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
HREG_LIB=$PWD/pcd_reg_hregnet_amd/ab_k3qw4.so timeout -k 10 120 python tools/op_bench.py knn --b 64 > $O/op_qw4.txt 2>&1 || { tail $O/op_qw4.txt; exit 1; }
timeout -k 10 120 python tools/op_bench.py knn --b 64 > $O/op_qw1.txt 2>&1 || { tail $O/op_qw1.txt; exit 1; }
cat $O/op_qw4.txt $O/op_qw1.txt | grep knn
bash tools/ab_lines.sh r5w_ab 2 "--steps 20 --warmup 5 --no-latency --no-eager-roofline" - lib:ab_k3qw4.so
