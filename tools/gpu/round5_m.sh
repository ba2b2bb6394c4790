#!/bin/bash
# GPU box (round 5): refreshed rocprofv3 evidence for the fp8 (mixed, spread conversions)
# and f16x3 (issue pattern) kernels as shipped at HEAD: kernel trace + FETCH/WRITE passes of
# their headline bench, then SQ counters on suite view 0.
set -o pipefail
bash profiles/collect.sh r5_fp8 fp8 || exit $?
bash profiles/collect.sh r5_f16x3 f16x3 || exit $?
bash tools/pmc_sq.sh fp8 view0 || exit $?
bash tools/pmc_sq.sh f16x3 view0 || exit $?
echo done
