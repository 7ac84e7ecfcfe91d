#!/bin/bash
# r6: configs[2] (B = 32) lines at merge 1 / 2 / 4 and the default line, one box
set -o pipefail
O=gpurun_out/r6b32; mkdir -p $O
export TMPDIR=/tmp
for m in 1 2 4; do
  timeout -k 10 400 python bench.py --batch 32 --steps 20 --warmup 5 --merge $m --no-cpu-baseline --no-latency --no-merge1 > $O/m$m.json 2> $O/m$m.err || { echo "m$m failed"; tail -5 $O/m$m.err; exit 1; }
  python -c "import json; d=json.load(open('$O/m$m.json')); print('B32 merge $m', d['value'], d['ms_per_step'], d['roofline']['frac'], d['config']['executor'][:60])"
done
timeout -k 10 400 python bench.py > $O/default.json 2> $O/default.err || { echo "default failed"; tail -5 $O/default.err; exit 1; }
python -c "import json; d=json.load(open('$O/default.json')); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('merge1'), d['cpu_baseline'] and d['cpu_baseline'].get('value'))"
timeout -k 10 400 python bench.py --model v2 > $O/v2.json 2> $O/v2.err || { echo "v2 failed"; tail -5 $O/v2.err; exit 1; }
python -c "import json; d=json.load(open('$O/v2.json')); print('v2', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('latency'), d['cpu_baseline'] and d['cpu_baseline'].get('value'))"
