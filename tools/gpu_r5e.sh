#!/bin/bash
# r5e: merged Model_V2 batches (--merge) x lanes x batched stage 1; configs[1] A/B vs the r5 start.
set -o pipefail
O=gpurun_out/r5e; mkdir -p $O; rm -f $O/*.json
export TMPDIR=/tmp
bash tools/ab_lines.sh fpsab4 1 "--steps 20 --warmup 5" "merged or model_v2 or fps or hier_feature" lib:ab_head.so || exit 1
run() {  # NAME SWITCHES ARGS
  HREG_SWITCHES=$2 timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline $3 > $O/v2_$1.json 2> $O/v2_$1.err || { tail $O/v2_$1.err; exit 1; }
  python -c "import json; d=json.load(open('$O/v2_$1.json')); print('v2 $1', d['value'], d['ms_per_step'], d['roofline']['frac'], (d.get('fps') or {}).get('level1', {}).get('us_per_iteration'))"
}
run m1l8bs V2_BATCH_STAGE1=1 "--merge 1 --lanes 8 --steps 16 --warmup 8"
run m2l4bs V2_BATCH_STAGE1=1 "--merge 2 --lanes 4 --steps 16 --warmup 8"
run m4l4bs V2_BATCH_STAGE1=1 "--merge 4 --lanes 4 --steps 48 --warmup 16"
run m4l4 "" "--merge 4 --lanes 4 --steps 48 --warmup 16"
run m4l2bs V2_BATCH_STAGE1=1 "--merge 4 --lanes 2 --steps 48 --warmup 16"
run m8l2bs V2_BATCH_STAGE1=1 "--merge 8 --lanes 2 --steps 48 --warmup 16"
run m4l8bs V2_BATCH_STAGE1=1 "--merge 4 --lanes 8 --steps 64 --warmup 32"
