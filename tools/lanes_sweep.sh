#!/bin/bash
# bench pairs/s vs graph lanes (batches in flight), same box
set -o pipefail
O=gpurun_out/lanes; mkdir -p $O
for l in "$@"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --lanes $l --steps 48 > $O/l$l.json 2> $O/l$l.err || { tail -3 $O/l$l.err; exit 1; }
  python -c "import json; d=json.load(open('$O/l$l.json')); print('lanes $l', d['value'], d['ms_per_step'])"
done
