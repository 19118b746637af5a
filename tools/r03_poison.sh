#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for m in 1 0; do
  CAPGEN_FWD_GRAPH=$m timeout -k 10 180 python -u tools/poison_probe.py > gpurun_out/poison_$m.log 2>&1 || { tail -20 gpurun_out/poison_$m.log; exit 1; }
  echo "== FWD_GRAPH=$m"; grep '^{' gpurun_out/poison_$m.log | cut -c1-900
done
