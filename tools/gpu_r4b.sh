# PMC passes, the DDP test, bench lines at the driver's --steps 20 and the default 48, and a
# kernel trace of the --steps 20 run for tools/timeline.py.  Outputs gpurun_out/r4b/.
set -o pipefail
O=gpurun_out/r4b; mkdir -p $O
export TMPDIR=/tmp
bash tools/pmc_r4.sh r4b/pmc || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k ddp > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python tools/replay_cost.py 20 48 > $O/replay.txt 2>&1 || { tail $O/replay.txt; exit 1; }; cat $O/replay.txt
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/b20.json 2> $O/b20.err || { tail $O/b20.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b48.json 2> $O/b48.err || { tail $O/b48.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
python - <<'P'
import json
for f in ("b20","b48"):
    d=json.load(open(f"gpurun_out/r4b/{f}.json")); print(f, d["value"], d["ms_per_step"], d["roofline"]["frac"])
P
python tools/timeline.py $(ls $O/trace/*kernel_trace.csv | head -1) | head -40
