#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/host
o=gpurun_out/host
CAPGEN_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-host-batches > $o/plain.json 2> $o/plain.err || { tail $o/plain.err; exit 1; }
CAPGEN_HOST_TIMING=1 CAPGEN_ZERO=2 timeout -k 10 200 python -u bench.py --dp1 --steps 60 --warmup 10 --no-cpu-baseline --no-host-batches > $o/dp1.json 2> $o/dp1.err || { tail $o/dp1.err; exit 2; }
for f in plain dp1; do echo "== $f"; cut -c1-200 $o/$f.json; python3 -c "
import json; d=json.load(open('$o/$f.json')); print('ms/step', d['ms_per_step'], 'host_issue', d['host_issue_ms_per_step'])"; grep "capgen host" $o/$f.err | tail -4; done
