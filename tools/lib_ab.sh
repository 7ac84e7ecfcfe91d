#!/bin/bash
# Paired bench lines of the current library against an alternative build (HREG_LIB=pcd_reg_hregnet_amd/ab_old.so,
# built from another tree and copied in by hand) after the GPU suite.  Outputs: gpurun_out/kab/.
set -o pipefail
O=gpurun_out/kab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > $O/new$r.json 2> $O/new$r.err || { echo bench failed; tail $O/new$r.err; exit 1; }
  HREG_LIB=$PWD/pcd_reg_hregnet_amd/ab_old.so timeout -k 10 200 python bench.py --no-cpu-baseline > $O/old$r.json 2> $O/old$r.err || { echo bench old failed; tail $O/old$r.err; exit 1; }
done
python - <<'P'
import json
for f in ("new1","old1","new2","old2"):
    d=json.load(open(f"gpurun_out/kab/{f}.json")); print(f, d["value"], d["ms_per_step"])
P
