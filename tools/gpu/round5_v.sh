#!/bin/bash
# GPU box (round 5): the bf16 kernel's weight stream with one M0 write per stage (four 1 KiB
# LDS-DMA pieces at instruction offsets 0..3072) against one per piece; bit-identity shows the
# offset applies to the LDS address too.
set -o pipefail
mkdir -p gpurun_out/r5v
timeout -k 10 300 python -u tools/kernel_lab.py --precision bf16 --rounds ${ROUNDS:-11} labn/b16/*.so \
  > gpurun_out/r5v/bf16_m0.json 2> gpurun_out/r5v/bf16_m0.err || { echo "lab rc=$?"; tail -5 gpurun_out/r5v/bf16_m0.err; exit 1; }
cat gpurun_out/r5v/bf16_m0.json
