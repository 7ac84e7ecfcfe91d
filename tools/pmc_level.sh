#!/bin/bash
# PMC passes over the standalone bf16x6 level kernels (tools/b6_experiment.py, variant 0):
# effective clock (GRBM_GUI_ACTIVE), MFMA busy, issue/wait split, instruction-cache counters.
set -o pipefail
O=gpurun_out/${1:-pmclvl}; mkdir -p $O
export TMPDIR=/tmp
rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o -E "^\s*(SQC?_[A-Z_]*(ICACHE|IFETCH|INST_LEVEL|LEVEL_INST)[A-Z_]*)" $O/avail.txt | sort -u > $O/icache_names.txt || true
[ "$2" = "mem" ] || timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --output-format csv -d $O/p1 -o run -- python3 tools/b6_experiment.py 0 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
[ "$2" = "mem" ] || echo pass1 done
if [ "$2" = "mem" ]; then
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum --output-format csv -d $O/p2 -o run -- python3 tools/b6_experiment.py 0 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
  echo pass2 done
fi
