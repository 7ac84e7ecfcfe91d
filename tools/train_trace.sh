#!/bin/bash
# Kernel trace of the captured training step (config 4 per-rank shape): where the step's time
# goes between kernels.   Outputs gpurun_out/TAG/ttrace.
set -o pipefail
TAG=${1:-r5t}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ttrace -o run -- \
  python3 bench.py --model train --steps 6 --warmup 2 --no-cpu-baseline > $O/ttrace.log 2>&1 || { echo ttrace failed; tail $O/ttrace.log; exit 1; }
tail -2 $O/ttrace.log
