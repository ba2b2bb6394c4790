#!/bin/bash
# GPU box (round 4): the whole -m gpu suite (verbose: the printed error figures are the
# record), smoke(), compiler-counted vs asm-counted LDS reads interleaved (bf16, fp8,
# f16x3), then the default bench line (two-view protocol).
set -o pipefail
OUT=gpurun_out/r4a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/gpu_suite.log 2>&1
rc=$?
echo "suite rc=$rc"; grep -E "^FAILED|passed|failed" $OUT/gpu_suite.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 120 tools/probes/x3_shape_probe 24 > $OUT/x3_shape_probe.txt 2>&1 || { echo "probe rc=$?"; tail -5 $OUT/x3_shape_probe.txt; exit 1; }
tail -6 $OUT/x3_shape_probe.txt
for p in bf16 fp8 f16x3; do
  timeout -k 10 200 python -u tools/kernel_lab.py --precision $p --rounds 11 nerf-dbr_amd/nerf_amd/_lib/libnerf_mi355x.so labx/libnerf_asmreads.so > $OUT/lab_$p.json 2> $OUT/lab_$p.err || { echo "lab $p rc=$?"; tail -5 $OUT/lab_$p.err; exit 1; }
done
cat $OUT/lab_*.json | grep -E "median_ms|max_abs" 
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
tail -c 400 $OUT/bench.json
