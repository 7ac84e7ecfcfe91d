#!/bin/bash
# Round-6 evidence on the final tree, each GPU step under its own time limit, chained.
#   bash tools/final_r6.sh TAG PARTS      (outputs gpurun_out/TAG/)
#   t: GPU suite (+ parity tables) + smoke      b: bench default line + the driver's --steps 20 line
#   x: kernel traces (graph + eager) + in-executor figure     p: FETCH / WRITE / MFMA PMC passes
#   v: Model_V2 line          r: training line           k: issue / wait counters (pmc_kernels)
#   q: training step kernel trace
set -o pipefail
TAG=${1:-r6f}; PARTS=${2:-tbx}
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
if [[ $PARTS == *t* ]]; then
  export HREG_PARITY_REPORT=$O/parity_gpu.txt; rm -f $HREG_PARITY_REPORT
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
  unset HREG_PARITY_REPORT
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
fi
if [[ $PARTS == *b* ]]; then
  timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err \
    || { echo bench20 failed; tail $O/bench20.err; exit 1; }
fi
if [[ $PARTS == *x* ]]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/xtrace -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-eager-roofline --no-latency --no-cpu-baseline --no-merge1 \
    > $O/xtrace.log 2>&1 || { echo xtrace failed; tail $O/xtrace.log; exit 1; }
  M=$(python -c "import json; print(json.load(open('$O/bench20.json'))['config'].get('merge', 1))" 2>/dev/null || echo 4)
  K=hregnet:b8:n16384:s20; [ "$M" -gt 1 ] && K=$K:m$M
  python tools/in_executor.py $O/xtrace $K $((20 / M)) $O/in_executor.json > $O/in_executor.log 2>&1 || tail $O/in_executor.log
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/xtrace_eager -o run -- \
    python3 bench.py --executor pipeline --steps 20 --warmup 4 --no-latency --no-cpu-baseline \
    > $O/xtrace_eager.log 2>&1 || { echo xtrace_eager failed; tail $O/xtrace_eager.log; exit 1; }
fi
if [[ $PARTS == *p* ]]; then
  B="python3 bench.py --steps 4 --warmup 4 --no-cpu-baseline --no-latency --executor pipeline"
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE \
    --output-format csv -d $O/mfma -o run -- $B > $O/mfma.log 2>&1 || { tail -5 $O/mfma.log; exit 1; }
fi
if [[ $PARTS == *v* ]]; then
  timeout -k 10 400 python bench.py --model v2 > $O/bench_v2.json 2> $O/bench_v2.err \
    || { echo v2 failed; tail $O/bench_v2.err; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/v2trace -o run -- \
    python3 bench.py --model v2 --steps 24 --warmup 12 --no-eager-roofline --no-latency --no-cpu-baseline \
    > $O/v2trace.log 2>&1 || { echo v2trace failed; tail $O/v2trace.log; exit 1; }
fi
if [[ $PARTS == *c* ]]; then  # configs[2]: batch 32 on one GPU, its line and kernel trace
  timeout -k 10 400 python bench.py --batch 32 --steps 20 --warmup 5 > $O/bench_b32.json 2> $O/bench_b32.err \
    || { echo b32 failed; tail $O/bench_b32.err; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b32trace -o run -- \
    python3 bench.py --batch 32 --steps 20 --warmup 5 --no-eager-roofline --no-latency --no-cpu-baseline --no-merge1 \
    > $O/b32trace.log 2>&1 || { echo b32trace failed; tail $O/b32trace.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b32trace_eager -o run -- \
    python3 bench.py --batch 32 --executor pipeline --steps 8 --warmup 2 --no-latency --no-cpu-baseline \
    > $O/b32trace_eager.log 2>&1 || { echo b32trace_eager failed; tail $O/b32trace_eager.log; exit 1; }
fi
if [[ $PARTS == *r* ]]; then
  timeout -k 10 300 python bench.py --model train --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_train.json 2> $O/bench_train.err \
    || { echo train failed; tail $O/bench_train.err; exit 1; }
fi
if [[ $PARTS == *q* ]]; then  # training step kernel trace
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/traintrace -o run -- \
    python3 bench.py --model train --steps 6 --warmup 2 --no-cpu-baseline \
    > $O/traintrace.log 2>&1 || { echo traintrace failed; tail $O/traintrace.log; exit 1; }
fi
if [[ $PARTS == *k* ]]; then
  bash tools/pmc_kernels.sh $TAG/pmck "--steps 4 --warmup 4" > /dev/null 2>&1 || echo "pmc_kernels failed"
fi
python - <<P
import json, os
for f in ("bench", "bench20", "bench_v2", "bench_train", "bench_b32"):
    p = "$O/" + f + ".json"
    if os.path.exists(p) and os.path.getsize(p):
        d = json.load(open(p)); r = d.get("roofline", {})
        print(f, d["value"], d["ms_per_step"], r.get("frac"), "inexec", (r.get("in_executor") or {}).get("frac"),
              "lat", (d.get("latency") or {}).get("graph_ms"),
              "fps", {k: (v or {}).get("us_per_iteration") for k, v in (d.get("fps") or {}).items() if k.startswith("level")})
P
