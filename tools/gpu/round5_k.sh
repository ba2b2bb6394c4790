#!/bin/bash
# GPU box (round 5): the bf16 kernel's next-tile sample prefetch (LDS-DMA) -- interleaved
# A/B against the previous build (labo/b16: timing and bit-identity), then the round-end
# rehearsal (round5_g.sh: suite, smoke, bench).
set -o pipefail
mkdir -p gpurun_out/r5k
timeout -k 10 300 python -u tools/kernel_lab.py --precision bf16 --rounds ${ROUNDS:-9} labo/b16/*.so \
  > gpurun_out/r5k/bf16_pf.json 2> gpurun_out/r5k/bf16_pf.err || { echo "lab rc=$?"; tail -5 gpurun_out/r5k/bf16_pf.err; exit 1; }
cat gpurun_out/r5k/bf16_pf.json
bash tools/gpu/round5_g.sh r5k
