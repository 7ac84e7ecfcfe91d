#!/bin/bash
# r5o: executor knobs on the merged line (--steps 20 --warmup 5: 4 batches per forward, 5 lanes):
# front streaming off, 8 hardware queues.
set -o pipefail
bash tools/ab_lines.sh r5o_ab 2 "--steps 20 --warmup 5 --no-latency --no-eager-roofline" - sw:FRONT_STREAM=0 env:GPU_MAX_HW_QUEUES=8
