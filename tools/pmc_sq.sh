#!/bin/bash
# SQ counter passes on one MLP kernel (800x600x128 renders through tools/kernel_lab.py):
# one rocprofv3 --pmc run per counter group, each under its own kill timeout.
#   tools/pmc_sq.sh <precision> [lab|view0|view1]   -> gpurun_out/sq_<precision>[_<pose>]/p{1,2}
set -u
PREC=${1:-bf16}
POSE=${2:-lab}
KRE="mlp_${PREC}_kernel"
case $PREC in bf16x3|f16x3) KRE="mlp_x3_kernel";; esac
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/sq_$PREC
[ "$POSE" != lab ] && OUT=${OUT}_$POSE
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for group in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $group -T --output-format csv --kernel-include-regex "$KRE" \
    -d "$OUT/p$i" -o run -- python3 $ROOT/tools/kernel_lab.py --precision $PREC --pose $POSE --rounds ${ROUNDS:-1} \
    $ROOT/nerf-dbr_amd/nerf_amd/_lib/libnerf_mi355x.so > "$OUT/p$i.log" 2>&1 || exit $?
done
echo "sq $PREC done"
