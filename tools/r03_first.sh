#!/bin/bash
# first engine of a process vs later engines (eager forward), per knob, 6 processes each
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/first.log
for kn in CAPGEN_WT=1 CAPGEN_X=0; do
 for rep in 1 2 3 4 5 6; do
  env CAPGEN_FWD_GRAPH=0 $kn timeout -k 10 180 python -u tools/poison_probe.py 2>&1 | grep '^{' | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$kn|', ' '.join(f\"{k}:{v['n']}\" for k,v in d.items() if isinstance(v,dict)))
" >> gpurun_out/first.log || { tail -5 gpurun_out/first.log; exit 1; }
 done
done
cat gpurun_out/first.log
