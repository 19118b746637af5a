#!/bin/bash
# true host enqueue cost: a short burst (3 steps) so the GPU queue never fills
set -o pipefail
mkdir -p gpurun_out/host
o=gpurun_out/host
for mode in dp1; do
  args="--steps 3 --warmup 10 --no-cpu-baseline --no-host-batches"
  [ $mode = dp1 ] && args="$args --dp1"
  for rep in 1 2 3; do
    env CAPGEN_ZERO=2 timeout -k 10 200 python -u bench.py $args > $o/$mode.json 2> $o/$mode.err || { tail $o/$mode.err; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('$o/$mode.json') if l.startswith('{')][-1]); print('$mode', 'ms/step', d['ms_per_step'], 'host_issue', d['host_issue_ms_per_step'])"
  done
done
