#!/bin/bash
# A/B on the GPU box: knn tests, then bench with HREG_KNND=0/1 and lanes 4/8.
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${1:-ab}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q -k knn --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for m in 0 1; do
  HREG_KNND=$m timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_knnd$m.json 2> $O/bench_knnd$m.err || { tail $O/bench_knnd$m.err; exit 1; }
  echo "knnd=$m $(python -c "import json;d=json.load(open('$O/bench_knnd$m.json'));print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --lanes 8 --steps 24 > $O/bench_l8.json 2> $O/bench_l8.err || { tail $O/bench_l8.err; exit 1; }
echo "lanes8 $(python -c "import json;d=json.load(open('$O/bench_l8.json'));print(d['value'], d['ms_per_step'])")"
