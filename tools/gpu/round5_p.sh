#!/bin/bash
# GPU box (round 5): what the f16x3 split's ReLU costs -- the shipped build (labn/x3/x3s2)
# against NERF_X3_SPLIT2 (hi toward zero, ReLU on the packed halves, lo by a clamped fma_mix:
# 4 VALU per two values instead of 5; max_abs_vs_first shows the rounding difference).
set -o pipefail
mkdir -p gpurun_out/r5p
timeout -k 10 500 python -u tools/kernel_lab.py --precision f16x3 --rounds ${ROUNDS:-7} labn/x3/*.so \
  > gpurun_out/r5p/x3_split2.json 2> gpurun_out/r5p/x3_split2.err || { echo "x3 lab rc=$?"; tail -5 gpurun_out/r5p/x3_split2.err; exit 1; }
cat gpurun_out/r5p/x3_split2.json
