#!/bin/bash
# round-4 check 6: A/B of the in-step dX tile choices (tools/dx_incontention_tune.py) against the table
set -o pipefail
O=gpurun_out/r04h
mkdir -p $O
F="1216,2048,512,0,1,8;1216,512,2048,0,1,24;1216,512,512,0,1,24;2304,2048,512,0,1,8;2304,512,1536,0,1,7;2304,512,2048,0,1,7;2304,512,512,0,1,12;2304,512,6144,0,1,7"
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-batches > $O/base$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/base$i.json'));print('table', d['ms_per_step'], d['dominant_kernel']['classes_us_per_step'])"
CAPGEN_GEMM_FORCE="$F" timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-batches > $O/dx$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/dx$i.json'));print('instep', d['ms_per_step'], d['dominant_kernel']['classes_us_per_step'])"
done
