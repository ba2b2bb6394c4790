#!/bin/bash
# GPU box: interleaved timing of the lab builds in labx/ (f16x3 render pass).
set -o pipefail
mkdir -p gpurun_out/lab
timeout -k 10 300 python -u tools/kernel_lab.py --precision f16x3 --rounds ${ROUNDS:-7} labx/*.so > gpurun_out/lab/lab.json 2> gpurun_out/lab/lab.err || { echo "lab rc=$?"; tail -5 gpurun_out/lab/lab.err; exit 1; }
cat gpurun_out/lab/lab.json
