# r6: weight-gradient GEMM through LDS (library A/B: ab_tnold.so = the dword-load kernel)
B="timeout -k 10 300 python bench.py --model train --steps 10 --warmup 2 --no-cpu-baseline"
mkdir -p gpurun_out/r6tn
for r in 1 2; do
  $B > gpurun_out/r6tn/new$r.json 2>gpurun_out/r6tn/new$r.err || exit 1
  HREG_LIB=pcd_reg_hregnet_amd/ab_tnold.so $B > gpurun_out/r6tn/old$r.json 2>gpurun_out/r6tn/old$r.err || exit 1
done
python tools/ab_lines_print.py gpurun_out/r6tn new1 old1 new2 old2
