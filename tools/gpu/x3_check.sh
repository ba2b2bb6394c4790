#!/bin/bash
# GPU box: split-precision parity tests (synthetic + Lego), then the x3 bench lines.
set -o pipefail
mkdir -p gpurun_out/x3
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16x3.py tests/test_gpu_lego.py -v -s --timeout 300 --timeout-method thread > gpurun_out/x3/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/x3/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for p in f16x3 bf16x3; do
  timeout -k 10 300 python -u bench.py --precision $p --no-extras --no-train --cpu-seconds 0 > gpurun_out/x3/bench_$p.json 2> gpurun_out/x3/bench_$p.err || { echo "bench $p rc=$?"; tail -20 gpurun_out/x3/bench_$p.err; exit 1; }
done
tail -c 300 gpurun_out/x3/bench_f16x3.json
if ls labx/*.so > /dev/null 2>&1; then
  timeout -k 10 300 python -u tools/kernel_lab.py --precision f16x3 --rounds 7 labx/*.so > gpurun_out/x3/lab.json 2> gpurun_out/x3/lab.err || { echo "lab rc=$?"; tail -5 gpurun_out/x3/lab.err; exit 1; }
  cat gpurun_out/x3/lab.json
fi
