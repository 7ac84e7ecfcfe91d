#!/bin/bash
# Bench A/B/C/A/B/C on one box: default tree vs the env assignments $1 and $2.
# Outputs: gpurun_out/${3:-abc}/.
set -o pipefail
O=gpurun_out/${3:-abc}; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for v in a b c; do
    case $v in a) E="";; b) E="$1";; c) E="$2";; esac
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline > $O/$v$i.json 2> $O/$v$i.err || { echo bench failed; tail $O/$v$i.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$v$i.json')); print('$v$i', d['value'], {k: v['avg_launch_us'] for k, v in d['roofline']['per_entry'].items() if 'group' in k})"
  done
done
