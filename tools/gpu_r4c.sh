# kernel trace of steady-state replays (tools/replay_cost.py) for tools/timeline.py
set -o pipefail
O=gpurun_out/r4c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/replay_cost.py 20 48 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
grep lanes $O/trace.log
python tools/timeline.py $(ls $O/trace/*kernel_trace.csv | head -1) > $O/timeline.txt
grep -A12 "x group_l1_6_kernel" $O/timeline.txt | grep -v "^segment.* 0 x" | head -80
