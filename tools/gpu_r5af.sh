#!/bin/bash
# r5af: the pruned level-1 FPS with the unique-maximum fast paths: parity (pruned kernel, all FPS, end to
# end, graphs), then paired lines (FPS_SORTED on / off) with the latency figure
set -o pipefail
O=gpurun_out/r5af; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -rf --timeout 120 --timeout-method thread \
  -k "fps_indexed" > $O/pytest_fi.log 2>&1 || { echo "fps_indexed tests failed"; tail -40 $O/pytest_fi.log; exit 1; }
tail -1 $O/pytest_fi.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_ops.py -m gpu -q -rf \
  --timeout 300 --timeout-method thread -k "fps or svd or graph or chain_fork or vs_oracle or reference_fixture or record or keypoint or lanes" \
  > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab_lines.sh r5af_ab 2 "--steps 20 --warmup 5 --no-eager-roofline" - sw:FPS_SORTED=0
