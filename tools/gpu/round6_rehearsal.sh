#!/bin/bash
# Round 6 rehearsal at HEAD, as the driver runs the round end: the whole -m gpu suite, smoke(), bench.
set -o pipefail
OUT=gpurun_out/${1:-r6rehearsal}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/gpu_suite.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?
grep -E "^FAILED|passed|failed" $OUT/gpu_suite.log | tail -5; tail -1 $OUT/smoke.log
python -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'])
for k,v in d.get('other_configs',{}).items(): print(k, v.get('rays_per_s'), v.get('mlp_kernel_ms'))" || true
exit $rc
