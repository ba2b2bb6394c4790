#!/bin/bash
# GPU box (round 5): the multi-GPU bench's per-rank bands rendered one at a time on this GPU
# (tools/band_scaling.py): the compute part of the N = 2/4/8 view time, per precision and for
# config 4's 64+128 hierarchical frame.
set -o pipefail
mkdir -p gpurun_out/r5q
for a in "--precision bf16" "--precision bf16 --importance 128" "--precision f16x3" "--precision fp8"; do
  timeout -k 10 240 python -u tools/band_scaling.py $a >> gpurun_out/r5q/band_scaling.jsonl 2>> gpurun_out/r5q/band_scaling.err \
    || { echo "band_scaling $a rc=$?"; tail -5 gpurun_out/r5q/band_scaling.err; exit 1; }
done
cat gpurun_out/r5q/band_scaling.jsonl
