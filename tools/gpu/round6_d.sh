#!/bin/bash
# Round 6 lab d: fp8 staging -- two chunks ahead, and pieces spread over the chunk's units (labf/).
set -o pipefail
mkdir -p gpurun_out/r6d
L="labf/libnerf_w8.so labf/libnerf_ship.so labf/libnerf_a2.so labf/libnerf_a2sp.so labf/libnerf_a2sp4.so"
timeout -k 10 240 python -u tools/kernel_lab.py --precision fp8 --rounds 11 --pose view0 $L > gpurun_out/r6d/lab_view0.json 2> gpurun_out/r6d/lab_view0.err
rc=$?
cat gpurun_out/r6d/*.json
exit $rc
