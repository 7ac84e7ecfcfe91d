# graph upload A/B at the driver's --steps 20 --warmup 5 (and 48), plus the capture / FPS tests
set -o pipefail
O=gpurun_out/r4d; mkdir -p $O; rm -f $O/*.json
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k "graph or capture or fps or trainer" > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2 3; do
  for v in on off; do
    S=""; [ $v = off ] && S="GRAPH_UPLOAD=0"
    HREG_SWITCHES=$S timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/s20_$v.$r.json 2> $O/s20_$v.$r.err || { tail $O/s20_$v.$r.err; exit 1; }
  done
done
python - <<'P'
import json, glob
for f in sorted(glob.glob("gpurun_out/r4d/*.json")):
    d = json.load(open(f)); print(f.split("/")[-1], d["value"], d["ms_per_step"])
P
