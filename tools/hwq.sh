#!/bin/bash
# hardware queues per process (GPU_MAX_HW_QUEUES, HIP default 4) for the graph executor's streams:
# bench lines at 4 / 8 / 16, 20 and 48 steps (gpurun_out/hwq/)
set -o pipefail
O=gpurun_out/hwq; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for q in ${QS:-4 8 16}; do
    for st in 20 48; do
      GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps $st --warmup 5 --no-cpu-baseline > $O/q$q.s$st.$r.json 2> $O/q$q.s$st.$r.err || { echo "q$q failed"; tail $O/q$q.s$st.$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/q$q.s$st.$r.json')); print('q$q s$st', d['value'], d['ms_per_step'])"
    done
  done
done
