#!/bin/bash
# round-4 check 14: weight-gradient group tile variant in the step (CAPGEN_DWG_VARIANT; 0 = tuned,
# variant 10 = 128x128 16 waves at C2).  The fused attention kernels hold 160-168 VGPRs per wave: beside
# a 16-wave dW workgroup (320 VGPRs per SIMD) only one fits per CU.
set -o pipefail
O=gpurun_out/r04x
mkdir -p $O
for i in 1 2; do
for v in 0 20 8 6 4; do
CAPGEN_DWG_VARIANT=$v timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host-batches > $O/v$v.$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/v$v.$i.json'));c=d['dominant_kernel']['classes_us_per_step'];print('dwg $v', d['ms_per_step'], c)"
done
done
