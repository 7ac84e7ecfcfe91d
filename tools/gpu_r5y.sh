#!/bin/bash
# r5y: kernel trace of the single-batch latency graph (1 lane, batch 8, replays separated by idle gaps)
set -o pipefail
O=gpurun_out/r5y; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/lt -o run -- python3 tools/latency_trace.py 8 \
  > $O/lt.log 2>&1 || { tail $O/lt.log; exit 1; }
grep "replay ms" $O/lt.log
python tools/timeline.py $(find $O/lt -name "*kernel_trace.csv" | head -1) group_l1_6_kernel --list > $O/timeline.txt
head -150 $O/timeline.txt
