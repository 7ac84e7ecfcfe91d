#!/bin/bash
# A/B of the working tree against another built tree (default _abhead, a git worktree of
# HEAD) on the same box: tests of the working tree, then the default bench of each tree,
# alternated.  Outputs: gpurun_out/$1/.
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${1:-abt}
OTHER=${OTHER:-_abhead}
mkdir -p $O
export TMPDIR=/tmp
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for t in . $OTHER; do
    n=$(basename $(cd $t && pwd))
    (cd $t && timeout -k 10 300 python bench.py --no-cpu-baseline) > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || { tail $O/bench_${n}_$r.err; exit 1; }
    echo "$t run $r: $(python -c "import json;d=json.load(open('$O/bench_${n}_$r.json'));r=d['roofline'];print(d['value'], r['avg_launch_us'], r['all_mfma']['ms_per_step'])")"
  done
done
