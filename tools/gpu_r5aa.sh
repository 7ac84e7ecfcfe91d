#!/bin/bash
# r5aa: WFPS levels 2/3 on two waves (HREG_FPS_WT1024 / WT512 = 128) with the leaner exchange
set -o pipefail
O=gpurun_out/r5aa; mkdir -p $O
export TMPDIR=/tmp
HREG_LIB=$PWD/pcd_reg_hregnet_amd/ab_wt128.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -rf \
  --timeout 120 --timeout-method thread -k "fps" > $O/pytest_wt128.log 2>&1 \
  || { echo "variant tests failed"; tail -30 $O/pytest_wt128.log; exit 1; }
tail -1 $O/pytest_wt128.log
bash tools/ab_lines.sh r5aa_ab 2 "--steps 20 --warmup 5 --no-eager-roofline" - lib:ab_wt128.so
