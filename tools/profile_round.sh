#!/bin/bash
# Measurement on the GPU box for round $1 (e.g. r1): the default bench line, the
# rocprofv3 kernel-trace stats of the same command, and (with "pmc") the
# FETCH_SIZE / WRITE_SIZE passes, each in its own run.  Outputs: gpurun_out/$1/.
set -e
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py > $O/trace.log 2>&1
# the same workload on the eager executor: kernel durations without the lane overlap,
# directly comparable with bench.py's HIP-event timings
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_eager -o run -- python3 bench.py --executor pipeline --no-cpu-baseline > $O/trace_eager.log 2>&1
if [ "$2" = "pmc" ]; then
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --executor pipeline > $O/fetch.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE --output-format csv -d $O/mfma -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --executor pipeline > $O/mfma.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --executor pipeline > $O/write.log 2>&1
fi
