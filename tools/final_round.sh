#!/bin/bash
# Round-end measurement in one GPU call: the gpu test suite, smoke(), the default bench
# line + rocprofv3 kernel-trace stats (graph and eager) + PMC traffic passes
# (tools/profile_round.sh), and the Model_V2 / training bench lines.  Outputs:
# gpurun_out/$1/.  Each GPU step has its own time limit; the first failure ends the call.
set -o pipefail
TAG=${1:-r1f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/profile_round.sh $TAG pmc || { echo "profile_round failed"; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline > $O/bench_v2.json 2> $O/bench_v2.err \
  || { echo "v2 bench failed"; tail -20 $O/bench_v2.err; exit 1; }
timeout -k 10 300 python bench.py --model train --steps 10 --warmup 2 > $O/bench_train.json \
  2> $O/bench_train.err || { echo "train bench failed"; tail -20 $O/bench_train.err; exit 1; }
python -c "import json
for f in ('bench_v2', 'bench_train'):
    d = json.load(open('$O/' + f + '.json')); print(f, d['value'], d['ms_per_step'])"
