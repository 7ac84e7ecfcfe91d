#!/bin/bash
# A/B of fps_blocks_kernel variants (libraries built by python -m pcd_reg_hregnet_amd.build --variant)
set -o pipefail
export TMPDIR=/tmp
for L in "$@"; do
  HREG_LIB=$PWD/pcd_reg_hregnet_amd/$L timeout -k 10 120 python tools/fps_blocks_time.py 65536 8 || exit 1
  HREG_LIB=$PWD/pcd_reg_hregnet_amd/$L timeout -k 10 120 python tools/fps_blocks_time.py 65536 64 || exit 1
done
