#!/bin/bash
# Collect the rocprofv3 evidence for one round on a GPU box:
#   profiles/collect.sh <round-tag>
# 1. kernel trace + stats of the default bench command (per-kernel durations);
# 2. two separate PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic of the same kernels.
# Outputs land in gpurun_out/prof_<tag>/ ; copy the summaries worth keeping into profiles/.
set -u
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BENCH="$ROOT/bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-error-check"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace" -o run \
  -- python3 $BENCH > "$OUT/trace_bench.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$OUT/pmc_fetch" -o run \
  -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-error-check > "$OUT/pmc_fetch.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$OUT/pmc_write" -o run \
  -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-error-check > "$OUT/pmc_write.log" 2>&1 || exit $?
echo "profiles in $OUT"
