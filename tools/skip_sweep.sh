#!/bin/bash
# Marginal cost of kernel families in the graph-pipelined bench step: the default bench
# line, then one bench line per HREG_SKIP set (those C-ABI entries not launched; outputs
# garbage -- timing analysis only).  Outputs: gpurun_out/skip/.
set -o pipefail
O=gpurun_out/skip; mkdir -p $O
run() {
  HREG_SKIP="$1" timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b.json 2> $O/b.err || { echo "fail $1"; tail -3 $O/b.err; return 0; }
  python -c "import json; d=json.load(open('$O/b.json')); print('%-60s %9.1f pairs/s %6.3f ms/step' % ('${1:-none}', d['value'], d['ms_per_step']))"
}
run ""
for s in "$@"; do run "$s"; done
run ""
