#!/bin/bash
# Round 6 lab e: fp8 with the next tile's fetch + encodings pipelined into the head units (labf/).
set -o pipefail
mkdir -p gpurun_out/r6e
L="labf/libnerf_ship.so labf/libnerf_pipe0.so labf/libnerf_pipe1.so"
timeout -k 10 240 python -u tools/kernel_lab.py --precision fp8 --rounds 11 --pose view0 $L > gpurun_out/r6e/lab_view0.json 2> gpurun_out/r6e/lab_view0.err && \
timeout -k 10 240 python -u tools/kernel_lab.py --precision fp8 --rounds 11 --pose lab $L > gpurun_out/r6e/lab_labpose.json 2> gpurun_out/r6e/lab_labpose.err
rc=$?
cat gpurun_out/r6e/*.json
exit $rc
