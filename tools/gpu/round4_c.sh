#!/bin/bash
# GPU box (round 4): the persistent fp8 kernel -- every fp8 GPU test, then an interleaved
# A/B against the previous (one workgroup per tile) build, labx/libnerf_head.so.
set -o pipefail
OUT=gpurun_out/r4c
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -k "fp8" -v -s --timeout 300 --timeout-method thread > $OUT/fp8_tests.log 2>&1
rc=$?
echo "fp8 tests rc=$rc"; grep -E "^FAILED|passed|failed" $OUT/fp8_tests.log | tail -8
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
# the split-bf16 unit built with -amdgpu-mfma-vgpr-form=1 (round 3 saw wrong sigmas with it
# while the fragment reads were asm with hand-counted waits; they are plain loads now)
NERF_MI355X_LIB=labx/libnerf_bf16x3vf.so timeout -k 10 600 python -u -m pytest tests -m gpu -k "bf16x3" -v -s \
  --timeout 300 --timeout-method thread > $OUT/bf16x3vf_tests.log 2>&1
rc2=$?
echo "bf16x3 vgpr-form tests rc=$rc2"; grep -E "^FAILED|passed|failed" $OUT/bf16x3vf_tests.log | tail -8
[ $rc2 -ne 0 ] && [ $rc2 -ne 1 ] && exit $rc2
timeout -k 10 200 python -u tools/kernel_lab.py --precision bf16x3 --rounds 7 \
  nerf-dbr_amd/nerf_amd/_lib/libnerf_mi355x.so labx/libnerf_bf16x3vf.so > $OUT/lab_bf16x3vf.json 2> $OUT/lab_bf16x3vf.err \
  || { echo "lab rc=$?"; tail -5 $OUT/lab_bf16x3vf.err; exit 1; }
cat $OUT/lab_bf16x3vf.json
for pose in view0 lab; do
  timeout -k 10 200 python -u tools/kernel_lab.py --precision fp8 --pose $pose --rounds 21 \
    nerf-dbr_amd/nerf_amd/_lib/libnerf_mi355x.so labx/libnerf_head.so > $OUT/lab_fp8_$pose.json 2> $OUT/lab_fp8_$pose.err \
    || { echo "lab rc=$?"; tail -5 $OUT/lab_fp8_$pose.err; exit 1; }
  cat $OUT/lab_fp8_$pose.json
done
timeout -k 10 150 tools/probes/x3_shape_probe 24 3 > $OUT/x3_shape_probe_power.txt 2>&1 || { echo "probe rc=$?"; tail -5 $OUT/x3_shape_probe_power.txt; exit 1; }
cat $OUT/x3_shape_probe_power.txt
