#!/bin/bash
# Counter passes on the bf16 MLP kernel (800x600x128, 2 renders): one rocprofv3 run per
# counter group (gfx950 SQ has 8 slots per pass).  Usage: tools/pmc_probe.sh <tag> "<counters...>" ...
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for group in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group -T --output-format csv --kernel-include-regex mlp_bf16 \
    -d "$OUT/p$i" -o run -- python3 $ROOT/tools/kernel_lab.py --rounds 1 \
    $ROOT/nerf-dbr_amd/nerf_amd/_lib/libnerf_mi355x.so > "$OUT/p$i.log" 2>&1 || exit $?
done
echo done
