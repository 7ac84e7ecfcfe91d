set -o pipefail
O=gpurun_out/ts; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_train_capture.py tests/test_gpu_train_graph.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
timeout -k 10 200 python bench.py --model train --steps 10 --warmup 2 > $O/two$r.json 2> $O/two$r.err || { echo bench failed; tail $O/two$r.err; exit 1; }
timeout -k 10 200 python -c "import sys; sys.argv=['bench.py','--model','train','--steps','10','--warmup','2']; from pcd_reg_hregnet_amd import trainer; trainer.TWO_STREAM=False; import bench; bench.main()" > $O/ser$r.json 2> $O/ser$r.err || { echo bench2 failed; tail $O/ser$r.err; exit 1; }
done
python - <<'P'
import json
for f in ("two1","ser1","two2","ser2"):
    d=json.load(open(f"gpurun_out/ts/{f}.json")); print(f, d["value"], d["ms_per_step"], d.get("loss_first_last"))
P
