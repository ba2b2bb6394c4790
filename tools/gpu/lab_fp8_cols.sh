#!/bin/bash
# GPU box: the two-column fp8 lab build (NERF_FP8_COLS=2) against the fp8 kernel before the
# knob (labx/a0_fp8old.so) and the default build after it (labx/a_base.so), interleaved; then
# the fp8 GPU tests on the default build and the SQ counters of the two-column build.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/lab_fp8c2
mkdir -p $OUT
timeout -k 10 300 python -u tools/kernel_lab.py --precision fp8 --rounds ${ROUNDS:-11} labx/*.so > $OUT/lab.json 2> $OUT/lab.err || { echo "lab rc=$?"; tail -5 $OUT/lab.err; exit 1; }
cat $OUT/lab.json
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_restated.py tests/test_gpu_parity.py -k "fp8" > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
export TMPDIR=/tmp
cd /tmp
i=0
for group in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $group -T --output-format csv --kernel-include-regex mlp_fp8_kernel \
    -d "$OUT/p$i" -o run -- python3 $ROOT/tools/kernel_lab.py --precision fp8 --rounds 1 \
    $ROOT/labx/b_fp8c2.so > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i rc=$?"; exit 1; }
done
echo "sq done"
