#!/bin/bash
# Round-2 evidence for the three MFMA MLP kernels: trace + HBM PMC passes of the
# headline bench (profiles/collect.sh) and SQ counter passes (tools/pmc_sq.sh).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
for p in bf16 fp8 bf16x3; do
  bash $ROOT/profiles/collect.sh r2_$p $p || exit $?
  bash $ROOT/tools/pmc_sq.sh $p || exit $?
done
echo "profiles done"
