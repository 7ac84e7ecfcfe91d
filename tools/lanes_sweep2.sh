#!/bin/bash
# bench pairs/s vs graph lanes at a given --steps ($1), same box: lanes in $2...
set -o pipefail
O=gpurun_out/lanes2s; mkdir -p $O
S=$1; shift
for l in "$@"; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --lanes $l --steps $S > $O/s${S}l$l.json 2> $O/s${S}l$l.err || { tail -3 $O/s${S}l$l.err; exit 1; }
  python -c "import json; d=json.load(open('$O/s${S}l$l.json')); print('steps $S lanes $l', d['value'], d['ms_per_step'], d['config']['executor'][-24:])"
done
