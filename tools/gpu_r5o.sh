#!/bin/bash
# r5o: executor knobs on the merged line (--steps 20 --warmup 5: 4 batches per forward, 5 lanes):
# front streaming off, 8 hardware queues.
set -o pipefail
bash tools/ab_lines.sh r5o_ab 2 "--steps 20 --warmup 5 --no-latency --no-eager-roofline" - sw:FRONT_STREAM=0 env:GPU_MAX_HW_QUEUES=8
timeout -k 10 300 python bench.py --model train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r5o_ab/bench_train.json 2> gpurun_out/r5o_ab/bench_train.err \
  || { echo train failed; tail gpurun_out/r5o_ab/bench_train.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r5o_ab/bench_train.json')); print('train', d['value'], d['ms_per_step'], d.get('loss_first_last'))"
