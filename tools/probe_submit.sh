#!/bin/bash
set -o pipefail
O=gpurun_out/r5l; mkdir -p $O
for L in 20 10; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-latency --no-eager-roofline --lanes $L > $O/b$L.json 2> $O/b$L.err || { tail $O/b$L.err; exit 1; }
python -c "import json; d=json.load(open('$O/b$L.json')); print('lanes $L', d['value'], d['ms_per_step'], 'host_submit_ms', d['host_submit_ms'], 'elapsed_ms', d['ms_per_step']*d['steps'])"
done
