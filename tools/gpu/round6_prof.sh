#!/bin/bash
# Round 6 evidence for a changed MLP kernel: rocprofv3 kernel trace + FETCH/WRITE passes of the
# headline bench at that precision (profiles/collect.sh), then the SQ passes on view 0.
#   tools/gpu/round6_prof.sh <precision> <tag>
set -o pipefail
PREC=${1:-fp8}
TAG=${2:-r6$PREC}
bash profiles/collect.sh $TAG $PREC && ROUNDS=3 bash tools/pmc_sq.sh $PREC view0
