#!/bin/bash
# GPU box: the whole -m gpu suite (verbose, printed errors kept), smoke(), the default bench line.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r3/gpu_suite.log 2>&1
rc=$?
echo "suite rc=$rc"; tail -5 gpurun_out/r3/gpu_suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/r3/smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/r3/bench.json 2> gpurun_out/r3/bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/r3/bench.err; exit 1; }
tail -c 400 gpurun_out/r3/bench.json
