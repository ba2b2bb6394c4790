#!/bin/bash
# GPU box (round 4): the split training forward with counted seam waits (4-slot ring) --
# every training GPU test, then an A/B kernel trace against HEAD's build and the
# timing-only build without the forward's rows.
set -o pipefail
OUT=$PWD/gpurun_out/r4k
mkdir -p $OUT
NERF_MI355X_LIB=$PWD/labx/libnerf_fwdcounted.so timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_bf16x3.py -q --timeout 200 --timeout-method thread > $OUT/train_tests.log 2>&1 || { echo "train tests rc=$?"; tail -30 $OUT/train_tests.log; exit 1; }
tail -1 $OUT/train_tests.log
cd /tmp
for v in head counted nostore; do
  lib=$GRAFT_REPO_ROOT/nerf-dbr_amd/nerf_amd/_lib/libnerf_mi355x.so
  lib=$GRAFT_REPO_ROOT/labx/libnerf_fwd$v.so
  NERF_MI355X_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/prof_$v -o run \
    -- python3 $GRAFT_REPO_ROOT/tools/train_profile.py 5 bf16x3 > $OUT/prof_$v.log 2>&1 || { echo "prof $v rc=$?"; tail -5 $OUT/prof_$v.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/prof_$v/run_kernel_stats.csv')):
    if 'x3' in r['Name'] or 'wgrad' in r['Name']: print('$v', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg')"
done
echo done
