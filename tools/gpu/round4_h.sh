#!/bin/bash
# GPU box (round 4): the split backward-data chain with and without its dZ row stores
# (timing-only ablation, labx/libnerf_bwdnostore.so), rocprofv3 kernel trace of
# tools/train_profile.py at precision bf16x3.
set -o pipefail
OUT=$PWD/gpurun_out/r4h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -q --timeout 200 --timeout-method thread > $OUT/train_tests.log 2>&1 || { echo "train tests rc=$?"; tail -20 $OUT/train_tests.log; exit 1; }
tail -1 $OUT/train_tests.log
cd /tmp
for v in default fwdplain; do
  lib=$GRAFT_REPO_ROOT/nerf-dbr_amd/nerf_amd/_lib/libnerf_mi355x.so
  [ $v != default ] && lib=$GRAFT_REPO_ROOT/labx/libnerf_$v.so
  NERF_MI355X_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/prof_$v -o run \
    -- python3 $GRAFT_REPO_ROOT/tools/train_profile.py 5 bf16x3 > $OUT/prof_$v.log 2>&1 || { echo "prof $v rc=$?"; tail -5 $OUT/prof_$v.log; exit 1; }
  python3 -c "
import csv
rows=list(csv.DictReader(open('$OUT/prof_$v/run_kernel_stats.csv')))
for r in rows:
    if 'bwd_x3' in r['Name'] or 'mlp_x3' in r['Name']: print('$v', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg')"
done
