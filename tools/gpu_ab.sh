#!/bin/bash
set -o pipefail
O=gpurun_out/r2b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -k "fine_head or nbr_head or fused_level" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
HREG_B6_HEADS=0 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_nob6.json 2> $O/bench_nob6.err || { echo bench failed; tail $O/bench_nob6.err; exit 1; }
python - <<'P'
import json
for f in ("bench", "bench_nob6"):
    d = json.load(open("gpurun_out/r2b/" + f + ".json"))
    print(f, d["value"], json.dumps(d["roofline"]["per_entry"]))
P
