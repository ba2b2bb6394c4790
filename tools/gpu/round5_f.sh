#!/bin/bash
# GPU box (round 5): interleaved A/B of the bf16 kernel against its one-wave-per-SIMD
# two-column form (NERF_BF16_WAVES=4, VGPR-form) with and without explicit issue patterns.
set -o pipefail
mkdir -p gpurun_out/r5f
timeout -k 10 300 python -u tools/kernel_lab.py --precision bf16 --rounds ${ROUNDS:-9} labb/*.so \
  > gpurun_out/r5f/bf16_w4.json 2> gpurun_out/r5f/bf16_w4.err || { echo "lab rc=$?"; tail -5 gpurun_out/r5f/bf16_w4.err; exit 1; }
cat gpurun_out/r5f/bf16_w4.json
