#!/bin/bash
# GPU tests, then the bench with HREG_COARSE_SPLIT=0/1 and the per-GEMM profile.
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${1:-ab}
mkdir -p $O
export TMPDIR=/tmp
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for m in 0 1; do
  env "${ABVAR:-HREG_COARSE_SPLIT}=$m" timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_cs$m.json 2> $O/bench_cs$m.err || { tail $O/bench_cs$m.err; exit 1; }
  echo "${ABVAR:-coarse_split}=$m $(python -c "import json;d=json.load(open('$O/bench_cs$m.json'));print(d['value'], d['ms_per_step'], d['roofline']['other_mfma_kernels']['gemm_nt_kernel'])")"
done
timeout -k 10 180 python tools/gemm_profile.py > $O/gemm.log 2>&1 || { tail $O/gemm.log; exit 1; }
cat $O/gemm.log
