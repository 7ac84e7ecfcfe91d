#!/bin/bash
# r5ac: sim_colmax with its row loads unrolled (bit-identical maxima): the similarity / CoarseReg /
# end-to-end tests, then three bench lines with the latency figure
set -o pipefail
O=gpurun_out/r5ac; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_ops.py -m gpu -q -rf \
  --timeout 300 --timeout-method thread -k "sim or coarse or chain_fork or graph_pipeline or vs_oracle or reference_fixture or head" \
  > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab_lines.sh r5ac_ab 3 "--steps 20 --warmup 5 --no-eager-roofline" -
