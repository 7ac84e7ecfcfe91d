#!/bin/bash
# One GPU call: the gpu suite, then Model_V2 (config 5, N = 65536) bench lines A/B/A/B with
# the level-1 kNN through the spatial index (default) and the full scan
# (HREG_SPATIAL_KNN_MAX=16384), then the training bench.  Outputs: gpurun_out/v2knn/.
set -o pipefail
O=gpurun_out/v2knn; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline > $O/v2_idx$r.json 2> $O/v2_idx$r.err \
    || { echo bench failed; tail $O/v2_idx$r.err; exit 1; }
  HREG_SPATIAL_KNN_MAX=16384 timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline \
    > $O/v2_scan$r.json 2> $O/v2_scan$r.err || { echo bench failed; tail $O/v2_scan$r.err; exit 1; }
done
timeout -k 10 300 python bench.py --model train --steps 10 --warmup 2 > $O/train.json 2> $O/train.err \
  || { echo train bench failed; tail $O/train.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --model v2 --no-cpu-baseline > $O/trace.log 2>&1 \
  || { echo prof failed; tail $O/trace.log; exit 1; }
python - "$O" <<'P'
import json, os, sys
for f in ("v2_idx1", "v2_scan1", "v2_idx2", "v2_scan2", "train"):
    d = json.load(open(os.path.join(sys.argv[1], f + ".json")))
    print(f, d["value"], d["ms_per_step"])
P
