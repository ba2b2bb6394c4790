#!/bin/bash
# GPU box (round 5): more explicit issue patterns, interleaved against the shipped ones --
# f16x3 (labn/x3: patterns 2 = shipped, 4, 5, 6) and the bf16 two-column kernel (labn/b16:
# 2 = shipped, 5, 6); mlp_x3.h / mlp_bf16.hip list the patterns.
set -o pipefail
mkdir -p gpurun_out/r5n
timeout -k 10 500 python -u tools/kernel_lab.py --precision f16x3 --rounds ${ROUNDS:-7} labn/x3/*.so \
  > gpurun_out/r5n/x3_sched.json 2> gpurun_out/r5n/x3_sched.err || { echo "x3 lab rc=$?"; tail -5 gpurun_out/r5n/x3_sched.err; exit 1; }
cat gpurun_out/r5n/x3_sched.json
timeout -k 10 300 python -u tools/kernel_lab.py --precision bf16 --rounds ${ROUNDS:-9} labn/b16/*.so \
  > gpurun_out/r5n/bf16_sched.json 2> gpurun_out/r5n/bf16_sched.err || { echo "bf16 lab rc=$?"; tail -5 gpurun_out/r5n/bf16_sched.err; exit 1; }
cat gpurun_out/r5n/bf16_sched.json
