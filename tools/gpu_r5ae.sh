#!/bin/bash
# r5ae: the pruned level-1 FPS with its Morton ranges interleaved over the waves: parity, then paired lines
set -o pipefail
O=gpurun_out/r5ae; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -rf --timeout 120 --timeout-method thread \
  -k "fps_indexed" > $O/pytest_fi.log 2>&1 || { echo "fps_indexed tests failed"; tail -40 $O/pytest_fi.log; exit 1; }
tail -1 $O/pytest_fi.log
bash tools/ab_lines.sh r5ae_ab 2 "--steps 20 --warmup 5 --no-eager-roofline" - sw:FPS_SORTED=0
