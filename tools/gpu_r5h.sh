#!/bin/bash
# r5h: the GPU suite (parity report), the level-3 tests on the 4-row-tile variant, then paired bench
# lines: the tree (level-2 batched x2 block, level-1 x2 block on one row tile) against each change
# reverted and against level 3 on 4 row tiles per wave.   Outputs gpurun_out/r5h/.
set -o pipefail
O=gpurun_out/r5h; mkdir -p $O
export TMPDIR=/tmp
export HREG_PARITY_REPORT=$O/parity_gpu.txt; rm -f $HREG_PARITY_REPORT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ${PYK:+-k "$PYK"} \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
unset HREG_PARITY_REPORT
HREG_LIB=$PWD/pcd_reg_hregnet_amd/ab_sj4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -m gpu -q -rf \
  --timeout 300 --timeout-method thread -k "two_tile or fused or vs_oracle or lanes_match" > $O/pytest_sj4.log 2>&1 \
  || { echo "sj4 pytest failed"; tail -30 $O/pytest_sj4.log; exit 1; }
tail -2 $O/pytest_sj4.log
bash tools/ab_lines.sh r5h_ab 2 "--no-latency" - lib:ab_x2b0.so lib:ab_l1x0.so lib:ab_sj4.so
