cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/l2pmc3 -o run -- python3 tools/op_bench.py l2 > gpurun_out/l2pmc3.log 2>&1
