#!/bin/bash
# round-4 check 13: decode A/B on the event fence scope (the generate path records no stream events:
# expect equal), then the un-profiled stamp timeline of the current build
set -o pipefail
O=gpurun_out/r04w
mkdir -p $O
for i in 1 2; do
for f in 1 0; do
CAPGEN_EVENT_FENCE=$f timeout -k 10 300 python -u tools/bench_generate.py > $O/gen$f.$i.json 2> $O/gen.err || { tail -20 $O/gen.err; exit 1; }
echo "fence $f"; cut -c1-200 $O/gen$f.$i.json
done
done
timeout -k 10 300 python -u tools/stamp_timeline.py --out $O/stamps > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
tail -3 $O/stamps.log
