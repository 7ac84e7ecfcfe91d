#!/bin/bash
# r5u: front-streaming copies as one foreach copy per lane: the executor tests, paired lines.
set -o pipefail
O=gpurun_out/r5u; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -m gpu -q -rf --timeout 300 --timeout-method thread \
  -k "graph or lanes or merged" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab_lines.sh r5u_ab 3 "--steps 20 --warmup 5 --no-latency --no-eager-roofline" - sw:FRONT_FOREACH=0
