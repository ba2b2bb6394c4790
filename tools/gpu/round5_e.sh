#!/bin/bash
# GPU box (round 5): interleaved A/B of the mixed fp8 kernel's conversion schedules (labf/).
set -o pipefail
mkdir -p gpurun_out/r5e
timeout -k 10 300 python -u tools/kernel_lab.py --precision fp8 --rounds ${ROUNDS:-9} labf/*.so \
  > gpurun_out/r5e/fp8_conv.json 2> gpurun_out/r5e/fp8_conv.err || { echo "lab rc=$?"; tail -5 gpurun_out/r5e/fp8_conv.err; exit 1; }
cat gpurun_out/r5e/fp8_conv.json
