#!/bin/bash
# GPU box (round 5): round-end rehearsal at HEAD -- the whole -m gpu suite, smoke(), the
# default bench line.
set -o pipefail
OUT=gpurun_out/${1:-r5g}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/gpu_suite.log 2>&1
rc=$?
echo "suite rc=$rc"; grep -E "^FAILED|passed|failed" $OUT/gpu_suite.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
tail -c 300 $OUT/bench.json; echo
