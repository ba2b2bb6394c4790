#!/bin/bash
# GPU box (round 4): the five tests fixed after r4a, then SQ counters of the three MFMA
# kernels on suite view 0 and view 1 (same binary and instruction stream, different operand
# values: is the MFMA pipe's idle time the schedule's or the power manager's?).
set -o pipefail
OUT=gpurun_out/r4b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_f16x3_range.py "tests/test_gpu_lego.py::test_lego_headline_full_frames_error_report" \
  tests/test_gpu_parity.py::test_bench_single_gpu_json_contract "tests/test_gpu_restated.py::test_encoding_fp32_large_coordinates" \
  > $OUT/fixed_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "^FAILED|passed|failed|f16x3 with|full frame" $OUT/fixed_tests.log | tail -12
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for p in fp8 bf16 f16x3; do
  r=40; [ $p = f16x3 ] && r=15
  for pose in view0 view1; do
    ROUNDS=$r timeout -k 10 280 bash tools/pmc_sq.sh $p $pose || { echo "pmc $p $pose rc=$?"; exit 1; }
    mv gpurun_out/sq_${p}_$pose $OUT/
  done
done
echo done
