#!/bin/bash
# GPU box (round 5): what the bf16 kernel's tile top costs -- interleaved timing of the
# shipped two-column build against timing-only ablations: the encodings of the first tile
# reused (PE_ONCE), the sample loads removed with the encodings still computed (NOFETCH), and
# the segment integral skipped (NOCOMPOSITE).
set -o pipefail
mkdir -p gpurun_out/r5j
timeout -k 10 300 python -u tools/kernel_lab.py --precision bf16 --rounds ${ROUNDS:-9} labo/b16/*.so \
  > gpurun_out/r5j/bf16_top.json 2> gpurun_out/r5j/bf16_top.err || { echo "lab rc=$?"; tail -5 gpurun_out/r5j/bf16_top.err; exit 1; }
cat gpurun_out/r5j/bf16_top.json
