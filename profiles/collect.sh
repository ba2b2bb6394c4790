#!/bin/bash
# Collect the rocprofv3 evidence for one round on a GPU box:
#   profiles/collect.sh <tag> [precision]
# The profiled command is the headline bench only (--no-extras --no-error-check,
# no CPU baseline), so every dispatch of the MLP kernel in it is a headline launch
# and the trace's average duration is directly comparable with bench.py's
# roofline.kernel_ms.
# 1. kernel trace + stats (per-kernel durations) — the JSON line it prints is kept;
# 2. two separate PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic of the same
#    command (MI355X_MICROARCH.md §HBM: one TCC group per pass).
# Outputs land in gpurun_out/prof_<tag>/ ; summarize.py copies the summaries into profiles/.
set -u
TAG=${1:-r01}
PREC=${2:-bf16}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS="--precision $PREC --cpu-seconds 0 --no-error-check --no-extras --no-train"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace" -o run \
  -- python3 $ROOT/bench.py --steps 10 --warmup 3 $ARGS > "$OUT/bench_under_rocprof.json" 2> "$OUT/trace.log" || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$OUT/pmc_fetch" -o run \
  -- python3 $ROOT/bench.py --steps 2 --warmup 1 $ARGS > "$OUT/pmc_fetch.log" 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$OUT/pmc_write" -o run \
  -- python3 $ROOT/bench.py --steps 2 --warmup 1 $ARGS > "$OUT/pmc_write.log" 2>&1 || exit $?
echo "$ARGS" > "$OUT/command.txt"
echo "profiles in $OUT"
