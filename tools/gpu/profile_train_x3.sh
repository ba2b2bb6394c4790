#!/bin/bash
# rocprofv3 kernel trace + stats of the training step with the split-bf16 forward
# (tools/train_profile.py 5 bf16x3), then FETCH_SIZE and WRITE_SIZE in separate passes.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
OUT=$ROOT/gpurun_out/prof_train_x3
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace" -o run \
  -- python3 $ROOT/tools/train_profile.py 5 bf16x3 > "$OUT/trace.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$OUT/pmc_fetch" -o run \
  -- python3 $ROOT/tools/train_profile.py 2 bf16x3 > "$OUT/pmc_fetch.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$OUT/pmc_write" -o run \
  -- python3 $ROOT/tools/train_profile.py 2 bf16x3 > "$OUT/pmc_write.log" 2>&1 || exit $?
echo "profiles in $OUT"
