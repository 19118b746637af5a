#!/bin/bash
# A/B an engine knob on one box: bash tools/ab_env.sh VAR v1 v2 ...  (two alternating rounds of
# a 100-step bench per value; prints ms/step).  Each bench run has its own time limit.
set -o pipefail
var=$1; shift
mkdir -p gpurun_out
for round in 1 2; do
  for v in "$@"; do
    env "$var=$v" timeout -k 10 120 python -u bench.py --steps 100 --no-cpu-baseline --no-host-batches > gpurun_out/ab.json 2> gpurun_out/ab.err \
      || { tail -20 gpurun_out/ab.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print('$var=$v', d['ms_per_step'], d['roofline']['scope'].split('step time ')[1][:10])"
  done
done
