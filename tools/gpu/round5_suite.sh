#!/bin/bash
# GPU box (round 5): the whole -m gpu suite (as the driver runs it at round end).
set -o pipefail
OUT=gpurun_out/${1:-r5suite}
mkdir -p $OUT
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/gpu_suite.log 2>&1
rc=$?
echo "suite rc=$rc"; grep -E "^FAILED|passed|failed" $OUT/gpu_suite.log | tail -12
exit $rc
