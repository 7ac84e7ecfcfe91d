#!/bin/bash
# One GPU call closing a session: smoke() and the headline bench line, then
# tools/train_check.sh (gpu suite, three training lines, training kernel profile).
# Outputs: gpurun_out/${1:-fin}/.
set -o pipefail
T=${1:-fin}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-60
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'])"
bash tools/train_check.sh $T
