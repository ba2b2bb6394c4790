#!/bin/bash
# GPU box: the whole -m gpu suite, then the default bench line (each under its own limit).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
rc=$?
echo "suite rc=$rc"; tail -3 gpurun_out/gpu_suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "bench rc=$?"
