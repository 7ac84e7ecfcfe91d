#!/bin/bash
# r5d: FPS temps storage / wide L1 geometry (configs[1] lines) and Model_V2 variants
# (batched stage 1, poll sleep, front streaming, lanes).  Outputs gpurun_out/r5d/.
set -o pipefail
O=gpurun_out/r5d; mkdir -p $O; rm -f $O/*.json
export TMPDIR=/tmp
bash tools/ab_lines.sh fpsab3 2 "--steps 20 --warmup 5" "fps or vs_oracle_lidar or model_v2_graph or hier_feature" lib:ab_head.so lib:ab_l1w.so || exit 1
run() {  # NAME LIB SWITCHES ARGS
  L=""; [ -n "$2" ] && L=$PWD/pcd_reg_hregnet_amd/$2
  HREG_LIB=$L HREG_SWITCHES=$3 timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline $4 > $O/v2_$1.json 2> $O/v2_$1.err || { tail $O/v2_$1.err; exit 1; }
  python -c "import json; d=json.load(open('$O/v2_$1.json')); print('v2 $1', d['value'], d['ms_per_step'], (d.get('fps') or {}).get('level1', {}).get('us_per_iteration'))"
}
run bs "" V2_BATCH_STAGE1=1 ""
run bs_s1 ab_sleep1.so V2_BATCH_STAGE1=1 ""
run bs_s4 ab_sleep4.so V2_BATCH_STAGE1=1 ""
run bsfs "" V2_BATCH_STAGE1=1,V2_FRONT_STREAM=1 ""
run bs8 "" V2_BATCH_STAGE1=1 "--lanes 8 --steps 16"
run bs8_s4 ab_sleep4.so V2_BATCH_STAGE1=1 "--lanes 8 --steps 16"
run bs8fs "" V2_BATCH_STAGE1=1,V2_FRONT_STREAM=1 "--lanes 8 --steps 16"
run bs16 "" V2_BATCH_STAGE1=1 "--lanes 16 --steps 16"
