#!/bin/bash
# r5q: Model_V2 at its new default (12 reference batches per forward): the line, a kernel trace,
# FETCH / WRITE PMC passes; HRegNet with the global-table level-1 kernel and level-2 WFPS on one
# wave (paired lines).
set -o pipefail
O=gpurun_out/r5q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline > $O/bench_v2.json 2> $O/bench_v2.err || { tail $O/bench_v2.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_v2.json')); print('v2', d['value'], d['ms_per_step'], d['config']['merge'], d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/v2trace -o run -- \
  python3 bench.py --model v2 --no-cpu-baseline --no-eager-roofline --no-latency > $O/v2trace.log 2>&1 || { echo v2trace failed; tail $O/v2trace.log; exit 1; }
B="python3 bench.py --model v2 --steps 24 --warmup 12 --no-cpu-baseline --no-latency --executor pipeline"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/v2fetch -o run -- $B > $O/v2fetch.log 2>&1 || { tail -5 $O/v2fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/v2write -o run -- $B > $O/v2write.log 2>&1 || { tail -5 $O/v2write.log; exit 1; }
HREG_LIB=$PWD/pcd_reg_hregnet_amd/ab_w1w.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -rf --timeout 120 \
  --timeout-method thread -k "fps" > $O/pytest_w1w.log 2>&1 || { echo "w1w fps tests failed"; tail -20 $O/pytest_w1w.log; exit 1; }
tail -1 $O/pytest_w1w.log
bash tools/ab_lines.sh r5q_ab 2 "--steps 20 --warmup 5 --no-eager-roofline" - sw:L1_LDS_MAX_N=0 lib:ab_w1w.so
