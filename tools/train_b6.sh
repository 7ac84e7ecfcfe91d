#!/bin/bash
# the training step's non-tall-skinny conv GEMMs on bf16x6 (TRAIN_B6) against
# the float64-replay gradient bars, then paired training bench lines (outputs gpurun_out/tb6/).
set -o pipefail
O=gpurun_out/tb6; mkdir -p $O
export TMPDIR=/tmp
HREG_SWITCHES=TRAIN_B6=1 timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k "train" > $O/pytest_b6.log 2>&1
rc=$?; tail -8 $O/pytest_b6.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2; do
  for v in base b6; do
    S=""; [ $v = b6 ] && S=TRAIN_B6=1
    HREG_SWITCHES=$S timeout -k 10 300 python bench.py --model train --steps 10 --warmup 2 --no-cpu-baseline > $O/$v.$r.json 2> $O/$v.$r.err || { echo "$v failed"; tail $O/$v.$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$v.$r.json')); print('$v', d['value'], d['ms_per_step'], d.get('loss_first_last'))"
  done
done
