#!/bin/bash
# SQ counter passes on the training step's MFMA kernels (tools/train_profile.py: main.py
# config): one rocprofv3 --pmc run per counter group, each under its own kill timeout.
#   tools/gpu/sq_train.sh [fp32|bf16x3]  -> gpurun_out/sq_train[_bf16x3]/p{1,2}
set -u
PREC=${1:-fp32}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
OUT=$ROOT/gpurun_out/sq_train
[ "$PREC" != fp32 ] && OUT=${OUT}_$PREC
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for group in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $group -T --output-format csv \
    --kernel-include-regex "wgrad_group_kernel|train_fwd_kernel|train_bwd_kernel|mlp_x3_kernel|train_bwd_x3_kernel" \
    -d "$OUT/p$i" -o run -- python3 $ROOT/tools/train_profile.py 2 $PREC > "$OUT/p$i.log" 2>&1 || exit $?
done
echo "sq train done"
