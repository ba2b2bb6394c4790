#!/bin/bash
# GPU box (round 5): bf16 two-column kernel ring geometry -- 16-unit chunks (half the seam
# barriers, 96 KiB ring) and a 6-slot ring of 8-unit chunks (seams wait for the stage three
# back), interleaved against the shipped 3 x 8-unit ring.
set -o pipefail
mkdir -p gpurun_out/r5l
timeout -k 10 300 python -u tools/kernel_lab.py --precision bf16 --rounds ${ROUNDS:-9} labo/b16/*.so \
  > gpurun_out/r5l/bf16_ring.json 2> gpurun_out/r5l/bf16_ring.err || { echo "lab rc=$?"; tail -5 gpurun_out/r5l/bf16_ring.err; exit 1; }
cat gpurun_out/r5l/bf16_ring.json
