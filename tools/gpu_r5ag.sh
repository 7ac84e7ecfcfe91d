#!/bin/bash
# r5ag: the pruned level-1 FPS's rank tree (HREG_FS_TREE) and unlikely-scan layout (HREG_FS_EXPECT): the
# FPS alone per library (with a bitwise check against the register kernel), three alternations
set -o pipefail
O=gpurun_out/r5ag; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for L in "" ab_fs00.so ab_fs10.so; do
    P=""; [ -n "$L" ] && P=$PWD/pcd_reg_hregnet_amd/$L
    HREG_LIB=$P timeout -k 10 120 python tools/fps_sorted_time.py >> $O/times.txt 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
  done
done
cat $O/times.txt
