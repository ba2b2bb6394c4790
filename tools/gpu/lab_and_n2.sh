#!/bin/bash
# GPU box: lab timing of labx/*.so, then the N=2 bench rehearsal on one GPU (gloo,
# two ranks sharing the device): exercises the N>1 line (dist record, self-checks).
set -o pipefail
mkdir -p gpurun_out/lab
bash tools/gpu/lab_only.sh || exit $?
NERF_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-grid --no-train \
  --cpu-seconds 0 > gpurun_out/lab/bench_n2_gloo.json 2> gpurun_out/lab/bench_n2_gloo.err || { echo "n2 rc=$?"; tail -20 gpurun_out/lab/bench_n2_gloo.err; exit 1; }
tail -c 1500 gpurun_out/lab/bench_n2_gloo.json
