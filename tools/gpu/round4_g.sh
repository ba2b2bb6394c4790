#!/bin/bash
# GPU box (round 4): per-kernel times of the training step, fp32 and bf16x3 (rocprofv3 kernel
# trace of tools/train_profile.py, main.py's configuration, profiled steps).
set -o pipefail
OUT=$PWD/gpurun_out/r4g
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for p in fp32 bf16x3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/prof_$p -o run \
    -- python3 $GRAFT_REPO_ROOT/tools/train_profile.py 5 $p > $OUT/prof_$p.log 2>&1 || { echo "prof $p rc=$?"; tail -5 $OUT/prof_$p.log; exit 1; }
  python3 -c "
import csv
rows=list(csv.DictReader(open('$OUT/prof_$p/run_kernel_stats.csv')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print('$p', r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg')"
done
