#!/bin/bash
# GPU box (round 5): rocprofv3 evidence for the round-5 bf16 kernel (two columns per wave) and
# SQ counters of it and of the f16x3 kernel with its issue pattern.
set -o pipefail
bash profiles/collect.sh r5_bf16 bf16 || exit $?
bash tools/pmc_sq.sh bf16 view0 || exit $?
bash tools/pmc_sq.sh f16x3 view0 || exit $?
echo done
