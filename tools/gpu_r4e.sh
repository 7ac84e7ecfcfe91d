# (1) the indexed-kNN pair variant: its kNN tests, then paired bench lines; (2) graph upload
# on / off at the driver's --steps 20 --warmup 5.  Outputs gpurun_out/r4e/.
set -o pipefail
O=gpurun_out/r4e; mkdir -p $O; rm -f $O/*.json
export TMPDIR=/tmp
V=$PWD/pcd_reg_hregnet_amd/ab_knnpair.so
HREG_LIB=$V timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k "knn or indexed or fixture or vs_oracle" > $O/pytest_pair.log 2>&1
rc=$?; tail -4 $O/pytest_pair.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k "graph or capture or fps or trainer" > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b48_base.$r.json 2> $O/e || { tail $O/e; exit 1; }
  HREG_LIB=$V timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b48_pair.$r.json 2> $O/e || { tail $O/e; exit 1; }
done
for v in PROBE_SKIP_GEMM=1 PROBE_SKIP_MLP=1; do
  HREG_SWITCHES=$v timeout -k 10 200 python bench.py --no-cpu-baseline > $O/probe_$v.json 2> $O/e || { tail $O/e; exit 1; }
done
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/s20_up.$r.json 2> $O/e || { tail $O/e; exit 1; }
  HREG_SWITCHES=GRAPH_UPLOAD=0 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/s20_noup.$r.json 2> $O/e || { tail $O/e; exit 1; }
done
timeout -k 10 200 python tools/op_bench.py knn > $O/knn_base.txt 2>&1 && HREG_LIB=$V timeout -k 10 200 python tools/op_bench.py knn > $O/knn_pair.txt 2>&1; tail -2 $O/knn_base.txt $O/knn_pair.txt
python - <<'P'
import json, glob
for f in sorted(glob.glob("gpurun_out/r4e/*.json")):
    d = json.load(open(f)); print(f.split("/")[-1], d["value"], d["ms_per_step"])
P
