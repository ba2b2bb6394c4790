#!/bin/bash
# Round 6 labs: fp8 two-column builds and f16x3 NODIR / PE_ONCE bounds, interleaved A/B (labf/).
set -o pipefail
mkdir -p gpurun_out/r6a
L="labf/libnerf_w8.so labf/libnerf_w4.so labf/libnerf_w4v.so labf/libnerf_w4s1.so labf/libnerf_w4s2.so labf/libnerf_w4s3.so labf/libnerf_w4vs2.so labf/libnerf_w4vs3.so"
X="labf/libnerf_x3ship.so labf/libnerf_x3nodir.so labf/libnerf_x3peonce.so labf/libnerf_x3both.so"
timeout -k 10 240 python -u tools/kernel_lab.py --precision fp8 --rounds 9 --pose view0 $L > gpurun_out/r6a/lab_view0.json 2> gpurun_out/r6a/lab_view0.err && \
timeout -k 10 240 python -u tools/kernel_lab.py --precision fp8 --rounds 9 --pose lab $L > gpurun_out/r6a/lab_labpose.json 2> gpurun_out/r6a/lab_labpose.err && \
timeout -k 10 300 python -u tools/kernel_lab.py --precision f16x3 --rounds 7 --pose view0 $X > gpurun_out/r6a/x3_view0.json 2> gpurun_out/r6a/x3_view0.err
rc=$?
cat gpurun_out/r6a/*.json
exit $rc
