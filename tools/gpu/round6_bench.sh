#!/bin/bash
# Round 6: smoke() and the default bench line, as the driver runs them at round end.
set -o pipefail
OUT=gpurun_out/${1:-r6bench}
mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?
tail -3 $OUT/smoke.log; python -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'])
oc=d.get('other_configs',{})
for k,v in oc.items(): print(k, v.get('rays_per_s'), v.get('pixels_over_1e-4'), v.get('mlp_frac_mixed_ceiling'), (v.get('vs_fp64') or {}))
print('cpu', (d.get('cpu_baseline') or {}).get('value'))" || true
exit $rc
