#!/bin/bash
# GPU box (round 5): f16x3 attribution -- interleaved timing of timing-only ablation builds of
# the shipped split-fp16 render kernel (labx/*.so: make variant_x3 with one NERF_X3_ABLATE_*
# item removed each, and all removed = the MFMA floor), then SQ counters of the mixed fp8
# kernel and of f16x3 on suite view 0.
set -o pipefail
mkdir -p gpurun_out/r5c
timeout -k 10 400 python -u tools/kernel_lab.py --precision f16x3 --rounds ${ROUNDS:-7} labx/*.so \
  > gpurun_out/r5c/x3_ablations.json 2> gpurun_out/r5c/x3_ablations.err || { echo "lab rc=$?"; tail -5 gpurun_out/r5c/x3_ablations.err; exit 1; }
cat gpurun_out/r5c/x3_ablations.json
timeout -k 10 300 python -u tools/kernel_lab.py --precision bf16 --rounds ${ROUNDS:-7} labb/*.so \
  > gpurun_out/r5c/bf16_sched.json 2> gpurun_out/r5c/bf16_sched.err || { echo "bf16 lab rc=$?"; tail -5 gpurun_out/r5c/bf16_sched.err; exit 1; }
cat gpurun_out/r5c/bf16_sched.json
bash tools/pmc_sq.sh fp8 view0 || exit $?
bash tools/pmc_sq.sh f16x3 view0 || exit $?
echo done
