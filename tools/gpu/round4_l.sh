#!/bin/bash
# GPU box (round 4, last): the shipped build with counted training seams -- the training and
# split-bf16 GPU tests, then the bench's training leg (stage times).
set -o pipefail
OUT=gpurun_out/r4l
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_bf16x3.py -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --width 160 --height 120 --spp 32 --cpu-seconds 0 --no-error-check --no-extras > $OUT/bench_train.json 2> $OUT/bench_train.err || { echo "bench rc=$?"; tail -20 $OUT/bench_train.err; exit 1; }
python -c "
import json; b=json.loads(open('$OUT/bench_train.json').read().strip().splitlines()[-1])['training']
print('fp32', b['ms_per_step']); x=b['bf16x3_forward']; print('bf16x3', x['ms_per_step'], x['stage_ms_rank0'])"
