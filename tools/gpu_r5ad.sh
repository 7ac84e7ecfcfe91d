#!/bin/bash
# r5ad: level-1 FPS over the spatial index's sorted copy with exact group pruning (FPS_SORTED) and the
# fused SVD + transform: parity tests first, then paired bench lines (FPS_SORTED on / off) with latency
set -o pipefail
O=gpurun_out/r5ad; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -rf --timeout 120 --timeout-method thread \
  -k "fps_indexed" > $O/pytest_fi.log 2>&1 || { echo "fps_indexed tests failed"; tail -40 $O/pytest_fi.log; exit 1; }
tail -1 $O/pytest_fi.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_ops.py -m gpu -q -rf \
  --timeout 300 --timeout-method thread -k "fps or svd or graph or chain_fork or vs_oracle or reference_fixture or record or keypoint" \
  > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab_lines.sh r5ad_ab 2 "--steps 20 --warmup 5 --no-eager-roofline" - sw:FPS_SORTED=0
