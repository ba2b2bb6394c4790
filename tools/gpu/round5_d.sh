#!/bin/bash
# GPU box (round 5): the split-fp16 kernel with its explicit issue pattern (NERF_X3_SCHED=2) --
# its gate tests, the bench line, rocprofv3 evidence for the fp8 (mixed) and f16x3 kernels,
# and the N = 2 self-launch rehearsal (bench.py --gpus 2 with no torchrun environment, gloo,
# both ranks on the one GPU).
set -o pipefail
OUT=gpurun_out/r5d
mkdir -p $OUT
PYT="python -u -m pytest -v -s --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_bf16x3.py tests/test_gpu_f16x3_range.py tests/test_gpu_lego.py \
  "tests/test_gpu_lego_c3.py::test_lego_c3_full_frames_vs_reference[f16x3]" > $OUT/x3_tests.log 2>&1
rc=$?
echo "x3 tests rc=$rc"; grep -E "^FAILED|passed|failed" $OUT/x3_tests.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
tail -c 300 $OUT/bench.json; echo
bash profiles/collect.sh r5_fp8 fp8 || exit $?
bash profiles/collect.sh r5_f16x3 f16x3 || exit $?
NERF_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-extras --no-train \
  --cpu-seconds 0 > $OUT/bench_n2_self_launch.json 2> $OUT/bench_n2_self_launch.err || { echo "n2 rc=$?"; tail -20 $OUT/bench_n2_self_launch.err; exit 1; }
tail -c 400 $OUT/bench_n2_self_launch.json; echo
echo done
