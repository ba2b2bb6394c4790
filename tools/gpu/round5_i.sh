#!/bin/bash
# GPU box (round 5): MFMA issue order at the power limit -- interleaved A/B of the bf16
# two-column kernel with each MFMA sharing an operand with its predecessor (order 1), the
# shipped order (0, one break per unit) and no sharing (2); f16x3 shipped vs order 1.
set -o pipefail
mkdir -p gpurun_out/r5i
timeout -k 10 300 python -u tools/kernel_lab.py --precision bf16 --rounds ${ROUNDS:-9} labo/b16/*.so \
  > gpurun_out/r5i/bf16_order.json 2> gpurun_out/r5i/bf16_order.err || { echo "lab rc=$?"; tail -5 gpurun_out/r5i/bf16_order.err; exit 1; }
cat gpurun_out/r5i/bf16_order.json
timeout -k 10 400 python -u tools/kernel_lab.py --precision f16x3 --rounds ${ROUNDS:-7} labo/x3/*.so \
  > gpurun_out/r5i/x3_order.json 2> gpurun_out/r5i/x3_order.err || { echo "x3 lab rc=$?"; tail -5 gpurun_out/r5i/x3_order.err; exit 1; }
cat gpurun_out/r5i/x3_order.json
