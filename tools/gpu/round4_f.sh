#!/bin/bash
# GPU box (round 4): the training backward-data chain on the split-bf16 MFMA -- every training
# GPU test, then the bench's training leg alone (fp32 and bf16x3 stage times).
set -o pipefail
OUT=gpurun_out/r4f
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -v -s --timeout 300 --timeout-method thread > $OUT/train_tests.log 2>&1
rc=$?
echo "train tests rc=$rc"; grep -E "^FAILED|passed|failed|\[train" $OUT/train_tests.log | tail -12
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --width 160 --height 120 --spp 32 --cpu-seconds 0 --no-error-check --no-extras > $OUT/bench_train.json 2> $OUT/bench_train.err || { echo "bench rc=$?"; tail -20 $OUT/bench_train.err; exit 1; }
python -c "
import json; b=json.loads(open('$OUT/bench_train.json').read().strip().splitlines()[-1])['training']
print('fp32', b['ms_per_step'], b['stage_ms_rank0']); x=b['bf16x3_forward']; print('bf16x3', x['ms_per_step'], x['stage_ms_rank0'], x.get('gemm_kernels_rank0'))"
