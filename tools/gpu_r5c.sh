#!/bin/bash
# r5c: FPS per-geometry pick/pairmask + FPS wave priority, configs[1] and Model_V2 lines.
set -o pipefail
O=gpurun_out/r5c; mkdir -p $O; rm -f $O/*.json
export TMPDIR=/tmp
bash tools/ab_lines.sh fpsab2 2 "--steps 20 --warmup 5" "fps or vs_oracle_lidar or fixture or hier_feature or rccl or model_v2_graph" lib:ab_head.so lib:ab_prio.so || exit 1
for v in base q8 prio bs bsprio bs8; do
  L=""; Q=""; S=""; A=""
  case $v in *prio*) L=$PWD/pcd_reg_hregnet_amd/ab_prio.so;; esac
  case $v in q8) Q=8;; esac
  case $v in bs*) S=V2_BATCH_STAGE1=1;; esac
  case $v in bs8) A="--lanes 8 --steps 16";; esac
  if [ -n "$Q" ]; then export GPU_MAX_HW_QUEUES=$Q; else unset GPU_MAX_HW_QUEUES; fi
  HREG_LIB=$L HREG_SWITCHES=$S timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline $A > $O/v2_$v.json 2> $O/v2_$v.err || { tail $O/v2_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/v2_$v.json')); print('v2 $v', d['value'], d['ms_per_step'], (d.get('fps') or {}).get('level1', {}).get('us_per_iteration'))"
done
