#!/bin/bash
# Issue / wait / unit-busy counters of every kernel of the eager pipelined bench, three
# separate --pmc passes (MI355X_MICROARCH.md: <= 8 SQ, 2 TA, 2 TD per pass; no trace domains).
#   bash tools/pmc_kernels.sh TAG ["BENCH ARGS"]   -> gpurun_out/TAG/{pa,pb,pc}, summary.txt
set -o pipefail
TAG=${1:-pmck}; BARGS=${2:-"--steps 3 --warmup 1"}
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py $BARGS --no-cpu-baseline --no-latency --executor pipeline"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O/pa -o run -- $B > $O/pa.log 2>&1 || { tail -5 $O/pa.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pb -o run -- $B > $O/pb.log 2>&1 || { tail -5 $O/pb.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc TD_TD_BUSY_sum TD_TC_STALL_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/pc -o run -- $B > $O/pc.log 2>&1 || { tail -5 $O/pc.log; exit 1; }
python3 tools/pmc_kernels.py $O > $O/summary.txt 2>&1; head -60 $O/summary.txt
