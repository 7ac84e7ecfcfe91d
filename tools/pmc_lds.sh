set -o pipefail
O=gpurun_out/pmclds; mkdir -p $O; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS --output-format csv -d $O/p -o run -- python3 tools/b6_experiment.py 0 > $O/p.log 2>&1 || { tail -5 $O/p.log; exit 1; }
echo ok
