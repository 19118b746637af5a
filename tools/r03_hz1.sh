#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for m in 1 0; do
  CAPGEN_FWD_GRAPH=$m timeout -k 10 120 python -u tools/hazard_first.py > gpurun_out/hz1_$m.log 2>&1 || { tail -20 gpurun_out/hz1_$m.log; exit 1; }
  echo "== FWD_GRAPH=$m"; grep -v amdgpu.ids gpurun_out/hz1_$m.log | head -40
done
