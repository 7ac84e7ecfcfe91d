#!/bin/bash
# Model_V2 bench: this tree vs the round-1 tree in _abhead/ (same box, same call)
set -o pipefail
O=$PWD/gpurun_out/v2r1; mkdir -p $O
timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline > $O/cur.json 2> $O/cur.err || { tail $O/cur.err; exit 1; }
(cd _abhead && timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline > $O/r1.json 2> $O/r1.err) || { tail $O/r1.err; exit 1; }
timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline > $O/cur2.json 2> $O/cur2.err || { tail $O/cur2.err; exit 1; }
python -c "
import json
for f in ('cur', 'r1', 'cur2'):
    d = json.load(open('$O/' + f + '.json')); print(f, d['value'], d['ms_per_step'])"
