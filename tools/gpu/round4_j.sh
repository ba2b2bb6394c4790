#!/bin/bash
# GPU box (round 4): the split-precision training step's evidence at HEAD -- kernel trace,
# FETCH_SIZE / WRITE_SIZE passes, SQ counter passes on its MFMA kernels, and the timing-only
# build without the forward's training rows (labx/libnerf_fwdnostore.so).
set -o pipefail
bash tools/gpu/profile_train_x3.sh || { echo "profile rc=$?"; exit 1; }
bash tools/gpu/sq_train.sh bf16x3 || { echo "sq rc=$?"; exit 1; }
OUT=$PWD/gpurun_out/r4j
mkdir -p $OUT
cd /tmp
for v in nostore default; do
  lib=$GRAFT_REPO_ROOT/nerf-dbr_amd/nerf_amd/_lib/libnerf_mi355x.so
  [ $v != default ] && lib=$GRAFT_REPO_ROOT/labx/libnerf_fwd$v.so
  NERF_MI355X_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/prof_$v -o run \
    -- python3 $GRAFT_REPO_ROOT/tools/train_profile.py 5 bf16x3 > $OUT/prof_$v.log 2>&1 || { echo "prof $v rc=$?"; tail -5 $OUT/prof_$v.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/prof_$v/run_kernel_stats.csv')):
    if 'x3' in r['Name'] or 'wgrad' in r['Name']: print('$v', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg')"
done
echo done
