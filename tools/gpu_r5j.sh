#!/bin/bash
# r5j: level/head kernel knobs -- level-1 younger waves at s_setprio 1, split-chain B split under
# the previous chunk's MFMAs -- as paired bench lines, and Model_V2 with the LDS-table level 1.
set -o pipefail
O=gpurun_out/r5j; mkdir -p $O
export TMPDIR=/tmp
HREG_LIB=$PWD/pcd_reg_hregnet_amd/ab_swp.so timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -m gpu -q -rf \
  --timeout 300 --timeout-method thread -k "two_tile or vs_oracle_lidar" > $O/pytest_swp.log 2>&1 \
  || { echo "swp pytest failed"; tail -30 $O/pytest_swp.log; exit 1; }
tail -1 $O/pytest_swp.log
bash tools/ab_lines.sh r5j_ab 2 "--no-latency" - lib:ab_l1prio.so lib:ab_swp.so || exit 1
bash tools/ab_lines.sh r5j_v2 2 "--model v2 --no-latency" - sw:L1_LDS_MAX_N=65536
