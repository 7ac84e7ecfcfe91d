#!/bin/bash
# r5ab: single-forward latency work (chain_fork: CoarseReg's kNNs beside the head products, its
# neighbour head beside the first similarity gather, one row tile per MLP-head workgroup): tests,
# paired lines (forks on / off), and the latency trace of the new chain.
set -o pipefail
O=gpurun_out/r5ab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_ops.py -m gpu -q -rf \
  --timeout 300 --timeout-method thread -k "row_tiles or chain_fork or graph or coarse or vs_oracle or reference_fixture or record or head" \
  > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab_lines.sh r5ab_ab 2 "--steps 20 --warmup 5 --no-eager-roofline" - sw:CHAIN_FORK=0 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/lt -o run -- python3 tools/latency_trace.py 8 \
  > $O/lt.log 2>&1 || { tail $O/lt.log; exit 1; }
grep "replay ms" $O/lt.log
python tools/timeline.py $(find $O/lt -name "*kernel_trace.csv" | head -1) group_l1_6_kernel --list > $O/timeline.txt
