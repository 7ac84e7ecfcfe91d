set -o pipefail
O=${GRAFT_REPO_ROOT}/gpurun_out/lanes; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do for L in 4 6 8; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --lanes $L --steps 24 > $O/l${L}_$r.json 2>/dev/null || exit 1
  echo "lanes $L run $r: $(python -c "import json;print(json.load(open('$O/l${L}_$r.json'))['value'])")"
done; done
