#!/bin/bash
# Wall-time cost of kernel families in the captured training step: bench lines with the named
# library entries run twice per call (HREG_SWITCHES=PROBE_TWICE=a+b, _lib.call), beside plain lines.
#   bash tools/train_probe.sh TAG ENTRY[,ENTRY] ...     (outputs gpurun_out/TAG/)
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
run() {  # run NAME PROBE
  HREG_SWITCHES=PROBE_TWICE=$(echo "$2" | tr , +) timeout -k 10 300 python bench.py --allow-probes --model train --steps 10 --warmup 2 --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { echo "$1 failed"; tail $O/$1.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$1.json')); print('$1', '$2', d['value'], d['ms_per_step'])"
}
run base0 ""
for p in "$@"; do run $(echo $p | tr ',' '+') $p; done
run base1 ""
