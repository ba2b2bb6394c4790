#!/bin/bash
# GPU box: the whole -m gpu suite (verbose), smoke(), the default bench line, the f16x3 bench line.
set -o pipefail
mkdir -p gpurun_out/fc
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/fc/gpu_suite.log 2>&1
rc=$?
echo "suite rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/fc/gpu_suite.log | tail -6
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fc/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/fc/smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/fc/bench.json 2> gpurun_out/fc/bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/fc/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --precision f16x3 --no-extras --no-train --cpu-seconds 0 > gpurun_out/fc/bench_f16x3.json 2> gpurun_out/fc/bench_f16x3.err || { echo "bench f16x3 rc=$?"; exit 1; }
tail -c 300 gpurun_out/fc/bench.json
