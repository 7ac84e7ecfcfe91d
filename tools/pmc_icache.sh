#!/bin/bash
# Instruction-cache PMC pass over a short graph-pipelined bench run (all kernels concurrent).
set -o pipefail
O=gpurun_out/${1:-icache}; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH --output-format csv -d $O/p -o run -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/p.log 2>&1 || { tail -5 $O/p.log; exit 1; }
echo done
