set -o pipefail
O=gpurun_out/hwq; mkdir -p $O; export TMPDIR=/tmp
for q in ${QS:-4 8 16}; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --no-cpu-baseline > $O/q$q.json 2> $O/q$q.err || { echo fail $q; tail -3 $O/q$q.err; exit 1; }
  python -c "import json; d=json.load(open('$O/q$q.json')); print('queues $q', d['value'], d['ms_per_step'])"
done
