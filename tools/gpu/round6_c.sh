#!/bin/bash
# Round 6 lab c: fp8 two-column attribution by interleaved ablations (timing-only builds in labf/).
set -o pipefail
mkdir -p gpurun_out/r6c
L="labf/libnerf_w8.so labf/libnerf_w4vs2.so labf/libnerf_abl_nodma.so labf/libnerf_abl_nobar.so labf/libnerf_abl_noread.so labf/libnerf_abl_noconv.so labf/libnerf_abl_peonce.so labf/libnerf_abl_all.so"
timeout -k 10 240 python -u tools/kernel_lab.py --precision fp8 --rounds 11 --pose view0 $L > gpurun_out/r6c/lab_view0.json 2> gpurun_out/r6c/lab_view0.err
rc=$?
cat gpurun_out/r6c/*.json
exit $rc
