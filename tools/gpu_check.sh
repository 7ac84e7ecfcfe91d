#!/bin/bash
# One GPU call: the gpu test suite, the GEMM tile A/B (HREG_GEMM_BIG), the default bench
# line.  Every GPU step under its own time limit; the first failure ends the call.
# Outputs: gpurun_out/$1/.
set -o pipefail
TAG=${1:-check}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
fi
for v in ${GEMM_VARIANTS:-0 1 2}; do
  HREG_GEMM_BIG=$v timeout -k 10 180 python tools/gemm_profile.py > $O/gemm_$v.log 2>&1 \
    || { echo "gemm_profile $v failed"; tail -20 $O/gemm_$v.log; exit 1; }
  echo "variant $v: $(tail -1 $O/gemm_$v.log)"
done
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err \
  || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
