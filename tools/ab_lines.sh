#!/bin/bash
# Paired bench lines, alternating the current tree and variants (HREG_LIB / HREG_SWITCHES), after
# an optional pytest -k selection.   bash tools/ab_lines.sh TAG REPS "BENCH ARGS" [TESTS|-] VARIANT...
#   VARIANT: lib:<file in pcd_reg_hregnet_amd/> | sw:NAME=V[,NAME=V] | env:NAME=V   (outputs gpurun_out/TAG/)
# Prints value, ms/step, roofline frac, single-batch latency and per-level FPS us/iteration.
set -o pipefail
TAG=$1; REPS=$2; BARGS=$3; TESTS=$4; shift 4
O=gpurun_out/$TAG; mkdir -p $O; rm -f $O/*.json
export TMPDIR=/tmp
if [ "$TESTS" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k "$TESTS" > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 $REPS); do
  for v in base "$@"; do
    L=""; S=""; E="AB_VARIANT=0"
    case $v in lib:*) L=$PWD/pcd_reg_hregnet_amd/${v#lib:};; sw:*) S=${v#sw:};; env:*) E=${v#env:};; esac
    tag=$(echo $v | tr ':=,/' '____')
    env $E HREG_LIB=$L HREG_SWITCHES=$S timeout -k 10 300 python bench.py --no-cpu-baseline $BARGS > $O/$tag.$r.json 2> $O/$tag.$r.err || { tail $O/$tag.$r.err; exit 1; }
  done
done
python - "$O" <<'P'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.load(open(f))
    fps = d.get("fps") or {}
    lat = d.get("latency") or {}
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["roofline"]["frac"], "lat", lat.get("graph_ms"),
          "fps", [fps.get(f"level{k}", {}).get("us_per_iteration") for k in (1, 2, 3)])
P
