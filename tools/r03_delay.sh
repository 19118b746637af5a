#!/bin/bash
# delay-injection diagnostic: divergence rate per knob setting (one process per run, eager forward)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/delay.log
run() { tag=$1; shift; for i in 1 2 3 4 5; do env CAPGEN_FWD_GRAPH=0 "$@" timeout -k 10 120 python -u tools/delay_probe.py 2>&1 | grep '^{' | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$tag', d['order'], ' '.join(f\"{k}:{v['n']}\" for k,v in d.items() if k.startswith(('g_','w_'))), (d.get('g_s1') or {}).get('first', [])[:1])
" >> gpurun_out/delay.log || { tail -5 gpurun_out/delay.log; exit 1; }; done; }
run default CAPGEN_X=0
run streams2 CAPGEN_STREAMS=2
run skip_adam CAPGEN_SKIP=32
run streams1 CAPGEN_STREAMS=1
cat gpurun_out/delay.log
