#!/bin/bash
# r5f: Model_V2 cluster-FPS spin budget / participant size; a V2 kernel trace of the merged
# executor; the configs[1] line.
set -o pipefail
O=gpurun_out/r5f; mkdir -p $O; rm -f $O/*.json
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b20.json 2> $O/b20.err || { tail $O/b20.err; exit 1; }
python -c "import json; d=json.load(open('$O/b20.json')); print('b20', d['value'], d['latency']['graph_ms'], [d['fps']['level%d' % k]['us_per_iteration'] for k in (1,2,3)])"
run() {  # NAME LIB SWITCHES ARGS
  L=""; [ -n "$2" ] && L=$PWD/pcd_reg_hregnet_amd/$2
  HREG_LIB=$L HREG_SWITCHES=$3 timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline $4 > $O/v2_$1.json 2> $O/v2_$1.err || { tail $O/v2_$1.err; exit 1; }
  python -c "import json; d=json.load(open('$O/v2_$1.json')); print('v2 $1', d['value'], d['ms_per_step'], d['roofline']['frac'], (d.get('fps') or {}).get('level1', {}).get('us_per_iteration'))"
}
A="--merge 8 --lanes 2 --steps 48 --warmup 16"
run m8 "" V2_BATCH_STAGE1=1 "$A"
run m8cap2k ab_cap2k.so V2_BATCH_STAGE1=1 "$A"
run m8s32 ab_s32.so V2_BATCH_STAGE1=1 "$A"
run m8l4 "" V2_BATCH_STAGE1=1 "--merge 8 --lanes 4 --steps 64 --warmup 32"
HREG_SWITCHES=V2_BATCH_STAGE1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/v2trace -o run -- \
  python3 bench.py --model v2 $A --no-cpu-baseline --no-eager-roofline > $O/v2trace.log 2>&1 || { echo v2trace failed; tail $O/v2trace.log; exit 1; }
python3 tools/timeline.py $O/v2trace/run_kernel_trace.csv fps_cluster_kernel > $O/v2timeline.txt 2>&1 || true
tail -30 $O/v2timeline.txt
