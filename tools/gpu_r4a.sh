# round-4 check: the GPU suite (parity tables to parity_gpu.txt) + paired bench lines of the
# current library against HREG_LIB=ab_old.so (the A/B variant)
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
export TMPDIR=/tmp HREG_PARITY_REPORT=$PWD/$O/parity_gpu.txt
rm -f $HREG_PARITY_REPORT
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --durations=30 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -45 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > $O/new$r.json 2> $O/new$r.err || { tail $O/new$r.err; exit 1; }
  HREG_LIB=$PWD/pcd_reg_hregnet_amd/ab_old.so timeout -k 10 200 python bench.py --no-cpu-baseline > $O/old$r.json 2> $O/old$r.err || { tail $O/old$r.err; exit 1; }
done
python - <<'P'
import json
for f in ("new1","old1","new2","old2"):
    d=json.load(open(f"gpurun_out/r4a/{f}.json")); print(f, d["value"], d["ms_per_step"], d["roofline"]["frac"])
P
exit $rc
