#!/bin/bash
# after the LayerNorm-backward fix: the round-3 final check, then the two-engine rates probe
# (tools/poison_probe.py, first engine vs later ones) in the default graph mode and eager
set -o pipefail
bash tools/r03_final.sh || exit $?
: > gpurun_out/first2.log
for kn in "CAPGEN_X=0" "CAPGEN_FWD_GRAPH=0"; do
 for rep in 1 2 3 4 5 6; do
  env $kn timeout -k 10 180 python -u tools/poison_probe.py 2>&1 | grep '^{' | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$kn|', ' '.join(f\"{k}:{v['n']}\" for k,v in d.items() if isinstance(v,dict)))
" >> gpurun_out/first2.log || { tail -5 gpurun_out/first2.log; exit 1; }
 done
done
cat gpurun_out/first2.log
