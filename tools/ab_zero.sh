set -o pipefail
O=gpurun_out/ab3; mkdir -p $O; export TMPDIR=/tmp
for v in base nogemm nomlp base2; do
  case $v in base|base2) E="";; nogemm) E="HREG_LIB=pcd_reg_hregnet_amd/libnogemm.so";; nomlp) E="HREG_LIB=pcd_reg_hregnet_amd/libnomlp.so";; esac
  env $E timeout -k 10 240 python bench.py --no-cpu-baseline > $O/$v.json 2> $O/$v.err || { echo fail $v; tail -3 $O/$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$v.json')); print('$v', d['value'], d['ms_per_step'])"
done
