#!/bin/bash
# Two-stream training step check (one GPU call): the training GPU tests, then paired bench lines
# of the captured step with the current switches and with one switch off ($1: python statement
# run before bench.main(), default trainer.TWO_STREAM=False).  Outputs: gpurun_out/ts/.
set -o pipefail
O=gpurun_out/ts; mkdir -p $O
export TMPDIR=/tmp
OFF=${1:-"from pcd_reg_hregnet_amd import trainer; trainer.TWO_STREAM=False"}
timeout -k 10 500 python -u -m pytest tests/test_gpu_train_capture.py tests/test_gpu_train_graph.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
timeout -k 10 200 python bench.py --model train --steps 10 --warmup 2 > $O/on$r.json 2> $O/on$r.err || { echo bench failed; tail $O/on$r.err; exit 1; }
timeout -k 10 200 python -c "import sys; sys.argv=['bench.py','--model','train','--steps','10','--warmup','2']; $OFF; import bench; bench.main()" > $O/off$r.json 2> $O/off$r.err || { echo bench2 failed; tail $O/off$r.err; exit 1; }
done
python - <<'P'
import json
for f in ("on1","off1","on2","off2"):
    d=json.load(open(f"gpurun_out/ts/{f}.json")); print(f, d["value"], d["ms_per_step"], d.get("loss_first_last"))
P
