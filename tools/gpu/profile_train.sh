#!/bin/bash
# rocprofv3 evidence for the training step (tools/train_profile.py: main.py config, 5 steps
# after 2 warm-up): kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate passes.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
OUT=$ROOT/gpurun_out/prof_train
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace" -o run \
  -- python3 $ROOT/tools/train_profile.py 5 > "$OUT/trace.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$OUT/pmc_fetch" -o run \
  -- python3 $ROOT/tools/train_profile.py 2 > "$OUT/pmc_fetch.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$OUT/pmc_write" -o run \
  -- python3 $ROOT/tools/train_profile.py 2 > "$OUT/pmc_write.log" 2>&1 || exit $?
echo "profiles in $OUT"
