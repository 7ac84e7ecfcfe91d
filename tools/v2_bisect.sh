#!/bin/bash
# Model_V2 bench across worktrees (bisecting a regression): ./, _abhead, _ab_<commit>...
set -o pipefail
O=$PWD/gpurun_out/v2bis; mkdir -p $O
for d in "$@"; do
  n=$(basename $d)
  (cd $d && timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline > $O/$n.json 2> $O/$n.err) || { tail $O/$n.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'])"
done
