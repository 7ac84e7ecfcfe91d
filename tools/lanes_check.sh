#!/bin/bash
# graph executor checks: the graph / pipeline GPU tests, then bench lines at several
# --steps / --lanes settings and the Model_V2 bench
set -o pipefail
O=gpurun_out/lanes2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "graph or pipeline or v2" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for a in "--steps 20 --warmup 5" "--steps 24" "--steps 48" "--steps 20 --warmup 5 --lanes 4"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline $a > $O/b.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$a', d['value'], d['ms_per_step'])"
done
timeout -k 10 200 python bench.py --model v2 --no-cpu-baseline > $O/v2.json 2> $O/v2.err || { tail -3 $O/v2.err; exit 1; }
python -c "import json; d=json.load(open('$O/v2.json')); print('v2', d['value'], d['ms_per_step'])"
