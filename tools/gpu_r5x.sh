#!/bin/bash
# r5x: the FPS exchange with fewer VALU per iteration (v_max_f32_dpp reductions, the slot select
# chain, the winning lane's own LDS write, all-lane candidate read): the FPS and end-to-end tests
# on the tree and on the macros-off variant, then paired bench lines with the latency figure.
set -o pipefail
O=gpurun_out/r5x; mkdir -p $O
export TMPDIR=/tmp
K="fps or wfps or vs_oracle or reference_fixture or randsample or keypoint"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -m gpu -q -rf \
  --timeout 300 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 \
  || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
HREG_LIB=$PWD/pcd_reg_hregnet_amd/ab_fpsmac0.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -rf \
  --timeout 120 --timeout-method thread -k "fps" > $O/pytest_mac0.log 2>&1 \
  || { echo "variant tests failed"; tail -30 $O/pytest_mac0.log; exit 1; }
tail -1 $O/pytest_mac0.log
bash tools/ab_lines.sh r5x_ab 2 "--steps 20 --warmup 5 --no-eager-roofline" - lib:ab_fpsmac0.so
