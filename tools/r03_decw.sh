#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do for cfg in "CAPGEN_DECODE_GROUP_LDS=1 CAPGEN_DECODE_GROUP_WAVES=1" "CAPGEN_DECODE_GROUP_LDS=0 CAPGEN_DECODE_GROUP_WAVES=1" "CAPGEN_DECODE_GROUP_LDS=1 CAPGEN_DECODE_GROUP_WAVES=2" "CAPGEN_DECODE_GROUP_LDS=0 CAPGEN_DECODE_GROUP_WAVES=2"; do
  env $cfg timeout -k 10 200 python -u tools/bench_generate.py --modes beam5 > gpurun_out/decw.log 2>&1 || { tail gpurun_out/decw.log; exit 1; }
  echo "$cfg $(grep '^{' gpurun_out/decw.log | cut -c100-160)"
done; done
