#!/bin/bash
# Round 6 lab b: fp8 two-column variants (issue patterns, two-ahead staging, prefetch 2), interleaved.
set -o pipefail
mkdir -p gpurun_out/r6b
L="labf/libnerf_w8.so labf/libnerf_w4vs2.so labf/libnerf_w4vs2a2.so labf/libnerf_w4vs1.so labf/libnerf_w4vs4.so labf/libnerf_w4vs2pf2.so labf/libnerf_w4vs2a2pf2.so labf/libnerf_w4vs4a2.so"
timeout -k 10 240 python -u tools/kernel_lab.py --precision fp8 --rounds 11 --pose view0 $L > gpurun_out/r6b/lab_view0.json 2> gpurun_out/r6b/lab_view0.err
rc=$?
cat gpurun_out/r6b/*.json
exit $rc
