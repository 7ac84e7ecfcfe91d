#!/bin/bash
# r5g: the GPU suite (32-slot cluster FPS default, batched V2 stage 1), Model_V2 lines around the
# new defaults, a V2 kernel trace and the V2 PMC traffic passes.   Outputs gpurun_out/r5g/.
set -o pipefail
O=gpurun_out/r5g; mkdir -p $O; rm -f $O/*.json
export TMPDIR=/tmp
export HREG_PARITY_REPORT=$O/parity_gpu.txt; rm -f $HREG_PARITY_REPORT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ${PYK:+-k "$PYK"} \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
unset HREG_PARITY_REPORT
run() {  # NAME LIB ARGS
  L=""; [ -n "$2" ] && L=$PWD/pcd_reg_hregnet_amd/$2
  HREG_LIB=$L timeout -k 10 300 python bench.py --model v2 --no-cpu-baseline $3 > $O/v2_$1.json 2> $O/v2_$1.err || { tail $O/v2_$1.err; exit 1; }
  python -c "import json; d=json.load(open('$O/v2_$1.json')); print('v2 $1', d['value'], d['ms_per_step'], d['roofline']['frac'], (d.get('fps') or {}).get('level1', {}).get('us_per_iteration'))"
}
run def "" ""
run def2 "" ""
run s16 ab_s16.so ""
run m8l4 "" "--merge 8 --lanes 4 --steps 64 --warmup 32"
run m16l2 "" "--merge 16 --lanes 2 --steps 64 --warmup 32"
run m4l4 "" "--merge 4 --lanes 4 --steps 48 --warmup 16"
run m4l2 "" "--merge 4 --lanes 2 --steps 48 --warmup 16"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/v2trace -o run -- \
  python3 bench.py --model v2 --no-cpu-baseline --no-eager-roofline > $O/v2trace.log 2>&1 || { echo v2trace failed; tail $O/v2trace.log; exit 1; }
B="python3 bench.py --model v2 --steps 16 --warmup 8 --no-cpu-baseline --executor pipeline"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/v2fetch -o run -- $B > $O/v2fetch.log 2>&1 || { tail -5 $O/v2fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/v2write -o run -- $B > $O/v2write.log 2>&1 || { tail -5 $O/v2write.log; exit 1; }
bash tools/pmc_kernels.sh pmck > /dev/null 2>&1 || echo "pmc failed"
head -30 gpurun_out/pmck/summary.txt
echo done
