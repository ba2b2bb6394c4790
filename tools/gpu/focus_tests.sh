#!/bin/bash
# GPU box: the split-precision, Lego, training and restated-kernel test files.
set -o pipefail
mkdir -p gpurun_out/ft
timeout -k 10 900 python -u -m pytest tests/test_gpu_bf16x3.py tests/test_gpu_lego.py tests/test_gpu_train.py tests/test_gpu_restated.py -v -s --timeout 300 --timeout-method thread > gpurun_out/ft/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/ft/tests.log | tail -8
exit $rc
