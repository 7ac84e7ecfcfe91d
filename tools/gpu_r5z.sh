#!/bin/bash
# r5z: quad maxima in the level-1 FPS scan (HREG_FPS_QUAD) and the single-forward side-stream forks
# (engine.chain_fork): tests on the tree and the level-2 quad variant, then paired bench lines with
# the latency figure (quads off / quads at level 2 too / forks off).
set -o pipefail
O=gpurun_out/r5z; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -m gpu -q -rf \
  --timeout 300 --timeout-method thread -k "fps or graph or chain_fork or vs_oracle or reference_fixture or keypoint" \
  > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
HREG_LIB=$PWD/pcd_reg_hregnet_amd/ab_fpsq16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -rf \
  --timeout 120 --timeout-method thread -k "fps" > $O/pytest_q16.log 2>&1 \
  || { echo "variant tests failed"; tail -30 $O/pytest_q16.log; exit 1; }
tail -1 $O/pytest_q16.log
bash tools/ab_lines.sh r5z_ab 2 "--steps 20 --warmup 5 --no-eager-roofline" - lib:ab_fpsq0.so lib:ab_fpsq16.so sw:CHAIN_FORK=0
