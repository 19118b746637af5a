#!/bin/bash
# round-4: weight-gradient group grid cap sweep (CAPGEN_DW_GRID; default = one workgroup per CU)
set -o pipefail
O=gpurun_out/r04k
mkdir -p $O
for i in 1 2; do
for g in 256 192 128 320; do
CAPGEN_DW_GRID=$g timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-batches > $O/g$g.$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/g$g.$i.json'));c=d['dominant_kernel']['classes_us_per_step'];print('grid $g', d['ms_per_step'], c['gemm dX'], c['gemm dW'])"
done
done
