# weight-gradient GEMM A/B (library A/B: ab_tnold.so = the build before the change)
#   bash tools/tn_ab.sh OUTDIR
O=gpurun_out/${1:-r6tn}
B="timeout -k 10 300 python bench.py --model train --steps 10 --warmup 2 --no-cpu-baseline"
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_graph.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  $B > $O/new$r.json 2>$O/new$r.err || exit 1
  HREG_LIB=pcd_reg_hregnet_amd/ab_tnold.so $B > $O/old$r.json 2>$O/old$r.err || exit 1
done
python tools/ab_lines_print.py $O new1 old1 new2 old2
