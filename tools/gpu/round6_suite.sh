#!/bin/bash
# GPU box (round 6): the -m gpu suite, or the part of it a -k expression selects ($2).
set -o pipefail
OUT=gpurun_out/${1:-r6suite}
mkdir -p $OUT
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread "${K[@]}" > $OUT/gpu_suite.log 2>&1
rc=$?
echo "suite rc=$rc"; grep -E "^FAILED|passed|failed" $OUT/gpu_suite.log | tail -12
exit $rc
