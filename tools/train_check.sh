#!/bin/bash
# One GPU call: the gpu suite, three training bench lines and the training-step kernel
# profile (rocprofv3 --kernel-trace --stats).  Outputs: gpurun_out/${1:-trc}/.
set -o pipefail
O=gpurun_out/${1:-trc}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --model train --steps 10 --warmup 2 > $O/t$r.json 2> $O/t$r.err \
    || { echo train bench failed; tail $O/t$r.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --model train --steps 10 --warmup 2 > $O/trace.log 2>&1 \
  || { echo prof failed; tail $O/trace.log; exit 1; }
python - "$O" <<'P'
import json, os, sys
for f in ("t1", "t2", "t3"):
    d = json.load(open(os.path.join(sys.argv[1], f + ".json")))
    print(f, d["value"], d["ms_per_step"])
P
