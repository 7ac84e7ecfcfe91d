#!/bin/bash
# r5i: Model_V2 evidence on the tree -- bench lines, a kernel trace, FETCH/WRITE PMC passes --
# then the issue / wait / unit-busy counters of configs[1]'s eager kernels.  Outputs gpurun_out/r5i/.
set -o pipefail
O=gpurun_out/r5i; mkdir -p $O; rm -f $O/*.json
export TMPDIR=/tmp
run() {  # NAME ARGS
  timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline $2 > $O/v2_$1.json 2> $O/v2_$1.err || { tail $O/v2_$1.err; exit 1; }
  python -c "import json; d=json.load(open('$O/v2_$1.json')); print('v2 $1', d['value'], d['ms_per_step'], d['roofline']['frac'], (d.get('fps') or {}).get('level1', {}).get('us_per_iteration'))"
}
run def ""
run def2 ""
run m8l4 "--merge 8 --lanes 4 --steps 64 --warmup 32"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/v2trace -o run -- \
  python3 bench.py --model v2 --no-cpu-baseline --no-eager-roofline --no-latency > $O/v2trace.log 2>&1 || { echo v2trace failed; tail $O/v2trace.log; exit 1; }
B="python3 bench.py --model v2 --steps 16 --warmup 8 --no-cpu-baseline --no-latency --executor pipeline"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/v2fetch -o run -- $B > $O/v2fetch.log 2>&1 || { tail -5 $O/v2fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/v2write -o run -- $B > $O/v2write.log 2>&1 || { tail -5 $O/v2write.log; exit 1; }
bash tools/pmc_kernels.sh pmck > /dev/null 2>&1 || echo "pmc failed"
head -40 gpurun_out/pmck/summary.txt
echo done
