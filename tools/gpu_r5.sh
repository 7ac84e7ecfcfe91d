#!/bin/bash
# Round-5 measurement, each GPU step under its own time limit, chained (the first failure ends
# the call).  bash tools/gpu_r5.sh TAG PARTS   (outputs gpurun_out/TAG/)
#   t: the GPU suite (+ parity tables)     b: the driver's bench line (--steps 20 --warmup 5)
#   x: rocprofv3 trace of the timed graph region -> in-executor figure (+ kernel stats)
#   v: Model_V2 line (config 5)            r: training line (config 4)
#   q: GPU_MAX_HW_QUEUES=2 refusal check (expects the guard's clean error)
set -o pipefail
TAG=${1:-r5a}
PARTS=${2:-tbx}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export TMPDIR=/tmp
if [[ $PARTS == *t* ]]; then
  export HREG_PARITY_REPORT=$O/parity_gpu.txt; rm -f $HREG_PARITY_REPORT
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
  unset HREG_PARITY_REPORT
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
fi
if [[ $PARTS == *b* ]]; then
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err \
    || { echo bench20 failed; tail $O/bench20.err; exit 1; }
fi
if [[ $PARTS == *x* ]]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/xtrace -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-eager-roofline --no-latency --no-cpu-baseline \
    > $O/xtrace.log 2>&1 || { echo xtrace failed; tail $O/xtrace.log; exit 1; }
  M=$(python -c "import json; print(json.load(open('$O/bench20.json'))['config'].get('merge', 1))" 2>/dev/null || echo 4)
  K=hregnet:b8:n16384:s20; [ "$M" -gt 1 ] && K=$K:m$M
  python tools/in_executor.py $O/xtrace $K $((20 / M)) $O/in_executor.json > $O/in_executor.log 2>&1 \
    || { tail $O/in_executor.log; }
fi
if [[ $PARTS == *v* ]]; then
  timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline > $O/bench_v2.json 2> $O/bench_v2.err \
    || { echo v2 failed; tail $O/bench_v2.err; exit 1; }
fi
if [[ $PARTS == *r* ]]; then
  timeout -k 10 300 python bench.py --model train --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_train.json 2> $O/bench_train.err \
    || { echo train failed; tail $O/bench_train.err; exit 1; }
fi
if [[ $PARTS == *q* ]]; then
  GPU_MAX_HW_QUEUES=2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    > $O/q2.json 2> $O/q2.err; echo "q2 rc=$?"; tail -2 $O/q2.err
fi
python - <<P
import json, os
for f in ("bench20", "bench_v2", "bench_train"):
    p = "$O/" + f + ".json"
    if os.path.exists(p) and os.path.getsize(p):
        d = json.load(open(p)); r = d.get("roofline", {})
        print(f, d["value"], d["ms_per_step"], r.get("frac"), "lat", (d.get("latency") or {}).get("graph_ms"),
              "fps", {k: (v or {}).get("us_per_iteration") for k, v in (d.get("fps") or {}).items() if k.startswith("level")})
P
