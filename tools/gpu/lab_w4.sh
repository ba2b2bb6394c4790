#!/bin/bash
# GPU box: interleaved timing of the two-column bf16 lab builds (labx/*.so), then the
# two SQ counter passes (tools/pmc_sq.sh groups) on labx/b_w4v.so.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/lab_w4
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/kernel_lab.py --precision bf16 --rounds ${ROUNDS:-11} labx/*.so > "$OUT/lab.json" 2> "$OUT/lab.err" || { echo "lab rc=$?"; tail -5 "$OUT/lab.err"; exit 1; }
cat "$OUT/lab.json"
export TMPDIR=/tmp
cd /tmp
i=0
for group in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $group -T --output-format csv --kernel-include-regex mlp_bf16_kernel \
    -d "$OUT/p$i" -o run -- python3 $ROOT/tools/kernel_lab.py --precision bf16 --rounds 1 \
    $ROOT/labx/b_w4v.so > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i rc=$?"; exit 1; }
done
echo "sq done"
