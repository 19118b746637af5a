#!/bin/bash
# round-4 check 8: A/B of the in-step forward tile choices (tools/dx_incontention_tune.py --fwd)
set -o pipefail
O=gpurun_out/r04r
mkdir -p $O
F="1216,512,2048,0,0,24;1216,512,512,0,0,24;2304,512,2048,0,0,12"
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-batches > $O/base$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/base$i.json'));c=d['dominant_kernel']['classes_us_per_step'];print('table', d['ms_per_step'], c['gemm fwd'], c['gemm dX'])"
CAPGEN_GEMM_FORCE="$F" timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-batches > $O/fwd$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/fwd$i.json'));c=d['dominant_kernel']['classes_us_per_step'];print('instep', d['ms_per_step'], c['gemm fwd'], c['gemm dX'])"
done
