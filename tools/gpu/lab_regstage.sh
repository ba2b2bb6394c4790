#!/bin/bash
# GPU box: register-staged weight streams (NERF_X3_REGSTAGE / NERF_BF16_REGSTAGE lab builds)
# against their LDS-DMA builds, interleaved: labx/a_x3base.so vs b_x3rs.so (f16x3 render
# pass), labx/c_base.so vs d_bf16rs.so (bf16).
set -o pipefail
OUT=gpurun_out/lab_rs
mkdir -p $OUT
timeout -k 10 300 python -u tools/kernel_lab.py --precision f16x3 --rounds ${ROUNDS:-9} labx/a_x3base.so labx/b_x3rs.so > $OUT/x3.json 2> $OUT/x3.err || { echo "x3 lab rc=$?"; tail -5 $OUT/x3.err; exit 1; }
cat $OUT/x3.json
timeout -k 10 300 python -u tools/kernel_lab.py --precision bf16 --rounds ${ROUNDS:-9} labx/c_base.so labx/d_bf16rs.so > $OUT/bf16.json 2> $OUT/bf16.err || { echo "bf16 lab rc=$?"; tail -5 $OUT/bf16.err; exit 1; }
cat $OUT/bf16.json
