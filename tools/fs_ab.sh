#!/bin/bash
# Front streaming (engine.FRONT_STREAM): the graph-executor tests, then paired bench lines at the
# driver's --steps 20 --warmup 5 and at 48 steps (outputs gpurun_out/fs/).
set -o pipefail
O=gpurun_out/fs; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -q -rf --timeout 300 --timeout-method thread -k "graph" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for v in 1 0; do
    HREG_SWITCHES=FRONT_STREAM=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/s20_fs$v.$r.json 2> $O/s20_fs$v.$r.err || { echo "fs=$v failed"; tail $O/s20_fs$v.$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/s20_fs$v.$r.json')); print('s20 fs=$v', d['value'], d['ms_per_step'])"
  done
done
for v in 1 0; do
  HREG_SWITCHES=FRONT_STREAM=$v timeout -k 10 300 python bench.py --no-cpu-baseline > $O/s48_fs$v.json 2> $O/s48_fs$v.err || { echo "fs=$v failed"; tail $O/s48_fs$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/s48_fs$v.json')); print('s48 fs=$v', d['value'], d['ms_per_step'])"
done
