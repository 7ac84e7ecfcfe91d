#!/bin/bash
# r5v: CoarseReg through layer-by-layer bf16x6 GEMMs (FUSED_COARSE=0) on the merged executor.
set -o pipefail
bash tools/ab_lines.sh r5v_ab 2 "--steps 20 --warmup 5 --no-latency" - sw:FUSED_COARSE=0
