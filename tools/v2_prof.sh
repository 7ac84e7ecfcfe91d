#!/bin/bash
set -o pipefail
O=gpurun_out/v2prof; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --model v2 --no-cpu-baseline > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
head -12 $O/trace/run_kernel_stats.csv | cut -c1-160
