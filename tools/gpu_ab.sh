# paired bench lines: the current library vs HREG_LIB=ab_old.so, alternating, $1 pairs
# (after the tests named in $2, a pytest -k expression; "" skips them).  Outputs gpurun_out/ab/.
set -o pipefail
O=gpurun_out/ab
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k "$2" > $O/pytest.log 2>&1
  rc=$?; tail -25 $O/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
for r in $(seq 1 ${1:-2}); do
  timeout -k 10 200 python bench.py --no-cpu-baseline > $O/new$r.json 2> $O/new$r.err || { tail $O/new$r.err; exit 1; }
  HREG_LIB=$PWD/pcd_reg_hregnet_amd/ab_old.so timeout -k 10 200 python bench.py --no-cpu-baseline > $O/old$r.json 2> $O/old$r.err || { tail $O/old$r.err; exit 1; }
done
python - <<'P'
import json, glob
for f in sorted(glob.glob("gpurun_out/ab/*.json")):
    d=json.load(open(f)); print(f.split("/")[-1], d["value"], d["ms_per_step"], d["roofline"]["frac"])
P
