#!/bin/bash
# Model_V2 bench A/B/A/B on one box: default tree vs the env assignment $1.
set -o pipefail
O=gpurun_out/${2:-v2ab}; mkdir -p $O
for i in 1 2; do
  for v in a b; do
    case $v in a) E="";; b) E="$1";; esac
    env $E timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline > $O/$v$i.json 2> $O/$v$i.err || { echo bench failed; tail $O/$v$i.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$v$i.json')); print('$v$i', d['value'], d['ms_per_step'])"
  done
done
