#!/bin/bash
# Per-round fixed cost of the graph executor: bench lines at --steps n (lanes = n, one round
# each), for a fit T(n) = a + b n of the round time (outputs gpurun_out/${1:-ls}/).
#   bash tools/lanes_sweep.sh [TAG] [n ...]
set -o pipefail
TAG=${1:-ls}; shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
NS=${@:-1 4 8 12 16 20 24 32 48}
for n in $NS; do
  timeout -k 10 300 python bench.py --steps $n --warmup 3 --no-cpu-baseline > $O/s$n.json 2> $O/s$n.err || { echo "steps $n failed"; tail $O/s$n.err; exit 1; }
  python -c "import json; d=json.load(open('$O/s$n.json')); print($n, d['value'], d['ms_per_step'], round(d['ms_per_step'] * $n, 3))"
done
