#!/bin/bash
# first engine of a process vs later engines, per setting, 7 processes each
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/first.log
for kn in "CAPGEN_FWD_GRAPH=0 CAPGEN_STREAMS=2 CAPGEN_COLSUM_SIDE=0" "CAPGEN_COLSUM_SIDE=0" "CAPGEN_X=0" "CAPGEN_FWD_GRAPH=0 CAPGEN_COLSUM_SIDE=0"; do
 for rep in 1 2 3 4 5 6 7; do
  env $kn timeout -k 10 180 python -u tools/poison_probe.py 2>&1 | grep '^{' | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$kn|', ' '.join(f\"{k}:{v['n']}\" for k,v in d.items() if isinstance(v,dict)))
" >> gpurun_out/first.log || { tail -5 gpurun_out/first.log; exit 1; }
 done
done
cat gpurun_out/first.log
