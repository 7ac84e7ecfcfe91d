#!/bin/bash
# r6: quick GPU check -- selected tests (pytest -k EXPR) then optional bench commands.
#   bash tools/r6_quick.sh TAG 'pytest -k expr' ['bench args' ...]
set -o pipefail
TAG=$1; K=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
if [ "$K" = all ]; then  # the whole GPU suite, with the parity tables
  export HREG_PARITY_REPORT=$O/parity_gpu.txt; rm -f $HREG_PARITY_REPORT
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
  unset HREG_PARITY_REPORT
  tail -3 $O/pytest.log
elif [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread -k "$K" \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
fi
i=0
for A in "$@"; do
  i=$((i+1))
  ENVS=(); ARGS="$A"
  while [[ $ARGS == HREG_* ]]; do ENVS+=("${ARGS%% *}"); [[ $ARGS == *" "* ]] && ARGS="${ARGS#* }" || ARGS=""; done
  env "${ENVS[@]}" timeout -k 10 400 python bench.py $ARGS > $O/bench$i.json 2> $O/bench$i.err || { echo "bench $i failed"; tail $O/bench$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench$i.json')); print('$A', '->', d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'), (d.get('fps') or {}).get('level1', {}).get('us_per_iteration') if isinstance(d.get('fps'), dict) else None)"
done
