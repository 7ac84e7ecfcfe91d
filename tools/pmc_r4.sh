#!/bin/bash
# PMC passes over a short eager pipelined bench run (each pass its own run):
# HBM traffic (FETCH_SIZE / WRITE_SIZE), the SQ issue / wait split, LDS / VMEM instruction mix.
# Outputs gpurun_out/$1/.
set -o pipefail
O=gpurun_out/${1:-pmc4}; mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --executor pipeline"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
echo fetch done
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
echo write done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC --output-format csv -d $O/sq -o run -- $B > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
echo sq done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O/sq2 -o run -- $B > $O/sq2.log 2>&1 || { tail -5 $O/sq2.log; exit 1; }
echo sq2 done
