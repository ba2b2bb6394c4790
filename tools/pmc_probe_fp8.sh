#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/pmc_fp8
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for group in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $group -T --output-format csv --kernel-include-regex mlp_fp8 \
    -d "$OUT/p$i" -o run -- python3 $ROOT/tools/kernel_lab.py --precision fp8 --rounds 1 \
    $ROOT/nerf-dbr_amd/nerf_amd/_lib/libnerf_mi355x.so > "$OUT/p$i.log" 2>&1 || exit $?
done
echo done
