#!/bin/bash
# round-4 check 19: the scheduling knobs re-swept on the final build (events without the system fence
# change what an extra fork / bucket edge costs): default, CAPGEN_BUCKET_BLOCKS=2, CAPGEN_STREAMS=2,
# CAPGEN_OVERLAP_DEC0=0, CAPGEN_PRIO=0 -- two alternating rounds
set -o pipefail
O=gpurun_out/r04ac
mkdir -p $O
for i in 1 2; do
for k in NONE CAPGEN_BUCKET_BLOCKS=2 CAPGEN_STREAMS=2 CAPGEN_OVERLAP_DEC0=0 CAPGEN_PRIO=0; do
if [ "$k" = NONE ]; then envs=""; else envs="$k"; fi
env $envs timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host-batches > $O/b.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/b.json'));print('$k', d['ms_per_step'])"
done
done
