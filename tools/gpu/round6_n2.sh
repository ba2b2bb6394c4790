#!/bin/bash
# Round 6: the N = 2 bench line on the one-GPU box (two ranks sharing the device over gloo,
# self-launched torchrun child), with the N > 1 CPU baseline and band-scaled traffic fields.
set -o pipefail
mkdir -p gpurun_out/r6n2
NERF_DIST_BACKEND=gloo timeout -k 10 900 python -u bench.py --gpus 2 --steps 3 --warmup 1 --cpu-seconds 12 --no-grid \
  > gpurun_out/r6n2/bench_n2.json 2> gpurun_out/r6n2/bench_n2.err
rc=$?
python -c "
import json; d=json.loads(open('gpurun_out/r6n2/bench_n2.json').read().strip().splitlines()[-1])
print(d['n_gpus'], d['value'], d['roofline']['traffic'], d['roofline']['traffic_source'][:80]); c=d['cpu_baseline']; print(c and (c['value'], c['cores'], c['n_gpus_protocol']))
print(d.get('self_check'), d.get('dist'))" || tail -20 gpurun_out/r6n2/bench_n2.err
exit $rc
