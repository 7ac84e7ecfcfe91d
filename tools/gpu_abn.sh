# bench lines of the current tree and variants, alternating, REPS rounds:
#   bash tools/gpu_abn.sh REPS STEPS [TESTS] VARIANT ...   (outputs gpurun_out/abn/)
# VARIANT: lib:<file in pcd_reg_hregnet_amd/> (HREG_LIB) or sw:NAME=V[,NAME=V] (HREG_SWITCHES);
# TESTS: a pytest -k expression run first ("-" for none)
set -o pipefail
O=gpurun_out/abn; mkdir -p $O; rm -f $O/*.json
export TMPDIR=/tmp
REPS=$1; STEPS=$2; TESTS=$3; shift 3
if [ "$TESTS" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k "$TESTS" > $O/pytest.log 2>&1
  rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
for r in $(seq 1 $REPS); do
  for v in base "$@"; do
    L=""; S=""
    case $v in lib:*) L=$PWD/pcd_reg_hregnet_amd/${v#lib:};; sw:*) S=${v#sw:};; esac
    tag=$(echo $v | tr ':=,/' '____')
    HREG_LIB=$L HREG_SWITCHES=$S timeout -k 10 200 python bench.py --no-cpu-baseline --steps $STEPS > $O/$tag.$r.json 2> $O/$tag.$r.err || { tail $O/$tag.$r.err; exit 1; }
  done
done
python - <<'P'
import json, glob
for f in sorted(glob.glob("gpurun_out/abn/*.json")):
    d = json.load(open(f))
    pe = d["roofline"]["per_entry"]
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["roofline"]["frac"],
          "fps_it_us", d.get("fps", {}).get("us_per_iteration"),
          {k.replace("hreg_", ""): v["avg_launch_us"] for k, v in pe.items()})
P
