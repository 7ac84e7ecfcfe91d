#!/bin/bash
# r5b: FPS pick A/B (+ tests), the counter list, a Model_V2 kernel trace.  Outputs gpurun_out/r5b/.
set -o pipefail
O=gpurun_out/r5b; mkdir -p $O
export TMPDIR=/tmp
bash tools/ab_lines.sh fpsab 2 "--steps 20 --warmup 5" "fps or rccl or vs_oracle_lidar or fixture" lib:ab_head.so lib:ab_pairmask.so || exit 1
timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/v2trace -o run -- \
  python3 bench.py --model v2 --steps 8 --warmup 4 --no-cpu-baseline --no-eager-roofline \
  > $O/v2trace.log 2>&1 || { echo v2trace failed; tail $O/v2trace.log; exit 1; }
python3 tools/timeline.py $(ls $O/v2trace/*kernel_trace.csv $O/v2trace/*/*kernel_trace.csv 2>/dev/null | head -1) fps_cluster_kernel > $O/v2timeline.txt 2>&1 || true
tail -40 $O/v2timeline.txt
