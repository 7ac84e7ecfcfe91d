#!/bin/bash
# One GPU call for an A/B: a pytest selection (-k $1), then the default bench line and the
# bench line with the env assignment $2 (e.g. HREG_B6_L1=0).  Outputs: gpurun_out/${3:-ab}/.
set -o pipefail
O=gpurun_out/${3:-ab}; mkdir -p $O
export TMPDIR=/tmp
if [ -n "$1" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$1" \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_a.json 2> $O/bench_a.err \
  || { echo bench failed; tail $O/bench_a.err; exit 1; }
if [ -n "$2" ]; then
  env $2 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_b.json 2> $O/bench_b.err \
    || { echo bench failed; tail $O/bench_b.err; exit 1; }
fi
python - "$O" <<'P'
import json, os, sys
for f in ("bench_a", "bench_b"):
    p = os.path.join(sys.argv[1], f + ".json")
    if os.path.exists(p):
        d = json.load(open(p))
        print(f, d["value"], json.dumps(d["roofline"]["per_entry"]))
P
