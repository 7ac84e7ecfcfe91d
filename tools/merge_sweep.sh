#!/bin/bash
# bench lines at one --steps over several --merge factors, two passes in mirrored order
#   bash tools/merge_sweep.sh OUTDIR STEPS WARMUP "M1 M2 ..."
set -o pipefail
O=gpurun_out/$1; S=$2; W=$3; MS=$4
mkdir -p $O
REV=$(echo $MS | tr ' ' '\n' | tac | tr '\n' ' ')
for pass in 1 2; do
  L=$MS; [ $pass = 2 ] && L=$REV
  for m in $L; do
    timeout -k 10 240 python bench.py --steps $S --warmup $W --merge $m --no-cpu-baseline --no-latency \
      --no-eager-roofline --no-merge1 > $O/m${m}_p$pass.json 2> $O/m${m}_p$pass.err \
      || { echo "merge $m failed"; tail -5 $O/m${m}_p$pass.err; exit 1; }
    python -c "import json; d=json.load(open('$O/m${m}_p$pass.json')); print('pass $pass merge $m', d['value'], d['config'].get('lanes', d['config']))"
  done
done
