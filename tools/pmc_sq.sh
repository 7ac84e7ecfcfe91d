#!/bin/bash
# One SQ counter pass (issue/wait breakdown) over a short eager bench run.
set -o pipefail
O=gpurun_out/${1:-sq}; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/sq -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --executor pipeline > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
echo done
