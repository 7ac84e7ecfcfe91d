# r6: the kNN lists' bitonic exchanges on DPP / permlane (library A/B: ab_knnold.so = ds_bpermute)
bash tools/r6_quick.sh r6kn "knn or vs_oracle or fixture or graph_pipeline_matches" || exit 1
timeout -k 10 120 python tools/knn_time.py > gpurun_out/r6kn/t_new.log 2>&1 && \
HREG_LIB=pcd_reg_hregnet_amd/ab_knnold.so timeout -k 10 120 python tools/knn_time.py > gpurun_out/r6kn/t_old.log 2>&1 || exit 1
cat gpurun_out/r6kn/t_new.log gpurun_out/r6kn/t_old.log
B="timeout -k 10 300 python bench.py --no-cpu-baseline --no-latency --no-merge1"
for r in 1 2; do
  $B > gpurun_out/r6kn/new$r.json 2>gpurun_out/r6kn/new$r.err || exit 1
  HREG_LIB=pcd_reg_hregnet_amd/ab_knnold.so $B > gpurun_out/r6kn/old$r.json 2>gpurun_out/r6kn/old$r.err || exit 1
done
python tools/ab_lines_print.py gpurun_out/r6kn new1 old1 new2 old2
