#!/bin/bash
# Round 6: the oracle's fp32 C3 chain on the GPU box's host CPU (another GEMM implementation)
# against the float64 truth, one view per call (tools/c3_truth_spread.py).  CPU only.
set -o pipefail
mkdir -p gpurun_out/r6spread
timeout -k 10 1150 python -u tools/c3_truth_spread.py gpurun_out/r6spread/spread_view$1.json $1
