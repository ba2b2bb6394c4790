#!/bin/bash
# GPU box (round 5, first run): the round-5 mixed fp8 kernel's tests first (new kernel), then
# the whole-frame C3 tests, then smoke() and the default bench line (the whole suite: round5_suite.sh).
set -o pipefail
OUT=gpurun_out/r5a
mkdir -p $OUT
PYT="python -u -m pytest -v -s --timeout 300 --timeout-method thread"
timeout -k 10 300 $PYT -x tests/test_gpu_restated.py -k "fp8 or low_gain" > $OUT/fp8_tests.log 2>&1
rc=$?
echo "fp8 tests rc=$rc"; grep -E "^FAILED|passed|failed|vs restatement|samples <=" $OUT/fp8_tests.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 $PYT tests/test_gpu_lego.py -k "fp8" > $OUT/fp8_lego.log 2>&1
rc=$?
echo "fp8 lego rc=$rc"; grep -E "^FAILED|passed|failed|lego" $OUT/fp8_lego.log | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 $PYT tests/test_gpu_lego_c3.py > $OUT/c3_tests.log 2>&1
rc=$?
echo "c3 tests rc=$rc"; grep -E "^FAILED|passed|failed|lego C3|pixels over|pixel \(" $OUT/c3_tests.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
tail -c 400 $OUT/bench.json
