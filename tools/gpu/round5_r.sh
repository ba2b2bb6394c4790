#!/bin/bash
# GPU box (round 5): the mixed fp8 kernel's fragment prefetch distance -- 2 units (NERF_FP8_PF=2)
# against the shipped 1, interleaved (max_abs_vs_first must be 0: same arithmetic).
set -o pipefail
mkdir -p gpurun_out/r5r
timeout -k 10 300 python -u tools/kernel_lab.py --precision fp8 --rounds ${ROUNDS:-9} labn/f8/*.so \
  > gpurun_out/r5r/fp8_pf.json 2> gpurun_out/r5r/fp8_pf.err || { echo "lab rc=$?"; tail -5 gpurun_out/r5r/fp8_pf.err; exit 1; }
cat gpurun_out/r5r/fp8_pf.json
