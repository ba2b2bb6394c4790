#!/bin/bash
# GPU box (round 4): the split-precision training step on ragged and tiny shapes.
set -o pipefail
OUT=gpurun_out/r4i
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -k "bf16x3" -v -s --timeout 200 --timeout-method thread > $OUT/train_x3.log 2>&1
rc=$?
grep -E "PASSED|FAILED|\[train|AssertionError|passed|failed" $OUT/train_x3.log | tail -30
exit $rc
