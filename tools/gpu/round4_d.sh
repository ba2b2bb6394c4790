#!/bin/bash
# GPU box (round 4): evidence at HEAD on the shipped Lego checkpoint -- rocprofv3 kernel
# trace + FETCH/WRITE passes for bf16, f16x3 and fp8 (profiles/collect.sh), SQ counters of
# the three kernels (2 s of renders each), then the x3 shape probe with activations that
# keep their size (power-limited regime).
set -o pipefail
OUT=gpurun_out/r4d
mkdir -p $OUT
for p in bf16 f16x3 fp8; do
  timeout -k 10 900 bash profiles/collect.sh r4_$p $p > $OUT/collect_$p.log 2>&1 || { echo "collect $p rc=$?"; tail -5 $OUT/collect_$p.log; exit 1; }
  tail -1 $OUT/collect_$p.log
done
for p in bf16 fp8 f16x3; do
  r=40; [ $p = f16x3 ] && r=15
  ROUNDS=$r timeout -k 10 280 bash tools/pmc_sq.sh $p || { echo "pmc $p rc=$?"; exit 1; }
done
timeout -k 10 150 tools/probes/x3_shape_probe 24 3 > $OUT/x3_shape_probe_power.txt 2>&1 || { echo "probe rc=$?"; tail -5 $OUT/x3_shape_probe_power.txt; exit 1; }
cat $OUT/x3_shape_probe_power.txt
timeout -k 10 400 python -u tools/kernel_lab.py --precision f16x3 --rounds 9 labx/libnerf_x3base.so labx/libnerf_x3spread.so \
  labx/libnerf_x3slots4.so > $OUT/lab_x3_spread.json 2> $OUT/lab_x3_spread.err || { echo "lab rc=$?"; tail -5 $OUT/lab_x3_spread.err; exit 1; }
cat $OUT/lab_x3_spread.json
