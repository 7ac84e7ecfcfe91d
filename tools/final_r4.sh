#!/bin/bash
# Round-4 measurement (each GPU step under its own time limit; the first failure ends the
# call), in two calls: PART a (tests, smoke, bench lines) and b (traces, PMC passes, V2 and
# training lines); both by default.  bash tools/final_r4.sh [TAG] [a|b|ab]
# Outputs gpurun_out/$1/ (default r4f):
#   pytest.log + parity_gpu.txt   the GPU suite with the parity tables (HREG_PARITY_REPORT)
#   smoke.log, bench.json (default 48 steps), bench20.json (the driver's --steps 20 --warmup 5)
#   trace/, trace_eager/          rocprofv3 --kernel-trace --stats of the graph and eager runs
#   fetch/, write/, mfma/         PMC passes (separate runs) over the eager pipelined run
#   bench_v2.json, bench_train.json
set -o pipefail
TAG=${1:-r4f}
PART=${2:-ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export TMPDIR=/tmp
if [[ $PART == *a* ]]; then
export HREG_PARITY_REPORT=$O/parity_gpu.txt
rm -f $HREG_PARITY_REPORT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
unset HREG_PARITY_REPORT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20.json 2> $O/bench20.err || { echo bench20 failed; tail $O/bench20.err; exit 1; }
fi
if [[ $PART == *b* ]]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_eager -o run -- python3 bench.py --executor pipeline --no-cpu-baseline > $O/trace_eager.log 2>&1 || { echo trace_eager failed; tail $O/trace_eager.log; exit 1; }
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --executor pipeline"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE --output-format csv -d $O/mfma -o run -- $B > $O/mfma.log 2>&1 || { tail -5 $O/mfma.log; exit 1; }
timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline > $O/bench_v2.json 2> $O/bench_v2.err || { echo v2 failed; tail $O/bench_v2.err; exit 1; }
timeout -k 10 300 python bench.py --model train --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_train.json 2> $O/bench_train.err || { echo train failed; tail $O/bench_train.err; exit 1; }
fi
python - <<P
import json, os
for f in ("bench", "bench20", "bench_v2", "bench_train"):
    if os.path.exists("$O/" + f + ".json"):
        d = json.load(open("$O/" + f + ".json")); print(f, d["value"], d["ms_per_step"], d.get("roofline", {}).get("frac"))
P
