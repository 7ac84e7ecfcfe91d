#!/bin/bash
# pairs/s when several 8-pair batches are merged into one forward (--batch), same box
set -o pipefail
O=gpurun_out/merge; mkdir -p $O
for cfg in "8 48" "48 8" "96 4" "192 2"; do
  set -- $cfg
  timeout -k 10 240 python bench.py --no-cpu-baseline --batch $1 --steps $2 > $O/b$1.json 2> $O/b$1.err || { tail -3 $O/b$1.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b$1.json')); print('batch $1 steps $2', d['value'], d['ms_per_step'], d['config']['executor'][-24:])"
done
