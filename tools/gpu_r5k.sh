#!/bin/bash
# r5k: level 3 in the pieces form (hreg_group_split6p_l3): its kernel test, the end-to-end oracle
# tests with it selected, then paired bench lines against the two-row-tile kernel.
set -o pipefail
O=gpurun_out/r5k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -m gpu -q -rf --timeout 300 --timeout-method thread \
  -k "pieces or two_tile" > $O/pytest_k.log 2>&1 || { echo "kernel test failed"; tail -40 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
export HREG_PARITY_REPORT=$O/parity_pieces.txt; rm -f $HREG_PARITY_REPORT
HREG_SWITCHES=L3_PIECES=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -m gpu -q -rf --timeout 300 \
  --timeout-method thread -k "vs_oracle or reference_fixture or lanes_match" > $O/pytest_e2e.log 2>&1 \
  || { echo "e2e failed"; tail -40 $O/pytest_e2e.log; exit 1; }
tail -1 $O/pytest_e2e.log
unset HREG_PARITY_REPORT
bash tools/ab_lines.sh r5k_ab 2 "--no-latency" - sw:L3_PIECES=1
