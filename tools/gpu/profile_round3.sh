#!/bin/bash
# GPU box: the training tests, then round-3 rocprofv3 evidence for the bf16 headline, the
# f16x3 gate path and fp8: kernel trace + stats and FETCH/WRITE passes (profiles/collect.sh),
# then the SQ counter passes (tools/pmc_sq.sh); every step under its own time limit.
set -o pipefail
mkdir -p gpurun_out/ft
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -q --timeout 300 --timeout-method thread > gpurun_out/ft/train_tests.log 2>&1 || { echo "train tests rc=$?"; tail -15 gpurun_out/ft/train_tests.log; exit 1; }
tail -1 gpurun_out/ft/train_tests.log
for p in bf16 f16x3 fp8; do
  bash profiles/collect.sh r3_$p $p > gpurun_out/collect_$p.log 2>&1 || { echo "collect $p rc=$?"; tail -5 gpurun_out/collect_$p.log; exit 1; }
  echo "collected $p"
done
for p in bf16 f16x3 fp8; do
  bash tools/pmc_sq.sh $p || { echo "sq $p rc=$?"; exit 1; }
done
