#!/bin/bash
# the graph-executor tests and two 20-step bench lines (outputs gpurun_out/fsc/)
set -o pipefail
O=gpurun_out/fsc; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -q -rf --timeout 300 --timeout-method thread -k "graph" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/s20.$r.json 2> $O/s20.$r.err || { tail $O/s20.$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/s20.$r.json')); print('s20', d['value'], d['ms_per_step'], d['config'].get('executor'))"
done
