#!/bin/bash
# GPU box: the fp8 packed-clamp conversion -- probe bit for bit, fp8 tests, interleaved
# timing against the previous build (labx/a_base.so), SQ counters of the new build.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/fp8pk
mkdir -p "$OUT"
timeout -k 10 120 python -u tools/probes/fp8_act_probe.py > "$OUT/probe.json" 2> "$OUT/probe.err" || { echo "probe rc=$?"; head -c 3000 "$OUT/probe.json"; tail -5 "$OUT/probe.err"; exit 1; }
grep -E '"(values|mismatches)"' "$OUT/probe.json"
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_restated.py tests/test_gpu_parity.py -k "fp8" > "$OUT/tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
timeout -k 10 300 python -u tools/kernel_lab.py --precision fp8 --rounds 11 labx/*.so > "$OUT/lab.json" 2> "$OUT/lab.err" || { echo "lab rc=$?"; tail -5 "$OUT/lab.err"; exit 1; }
cat "$OUT/lab.json"
timeout -k 10 300 bash tools/pmc_sq.sh fp8 || { echo "sq rc=$?"; exit 1; }
