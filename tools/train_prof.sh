#!/bin/bash
# Training step: bench lines and a kernel trace (outputs gpurun_out/${1:-tp}/).
#   bash tools/train_prof.sh [TAG] [LIB...]   LIB: extra libraries (HREG_LIB) for paired lines
set -o pipefail
TAG=${1:-tp}; shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --model train --steps 10 --warmup 2 --no-cpu-baseline > $O/train.json 2> $O/train.err || { echo train failed; tail $O/train.err; exit 1; }
for L in "$@"; do
  t=$(basename $L .so)
  HREG_LIB=$PWD/pcd_reg_hregnet_amd/$L timeout -k 10 300 python bench.py --model train --steps 10 --warmup 2 --no-cpu-baseline > $O/train_$t.json 2> $O/train_$t.err || { echo train $t failed; tail $O/train_$t.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --model train --steps 10 --warmup 2 --no-cpu-baseline > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
python - <<P
import json, glob
for f in sorted(glob.glob("$O/train*.json")):
    d = json.load(open(f)); print(f, d["value"], d["ms_per_step"], d.get("loss_first_last"))
P
