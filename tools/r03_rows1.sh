#!/bin/bash
# LayerNorm backward at one row per wave: the two strict bit-exactness tests that were xfail,
# then bench A/B against two rows per wave
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 180 --timeout-method thread -rxX \
  tests/test_gpu_hazard.py::test_side_stream_delay_leaves_bf16_results_bit_identical \
  tests/test_gpu_parity.py::test_bf16_weight_gradients_bit_reproducible_multistream \
  tests/test_gpu_parity.py::test_bf16_weight_gradients_bit_reproducible > gpurun_out/xf.log 2>&1 || { echo tests-failed; tail -30 gpurun_out/xf.log; exit 1; }
tail -8 gpurun_out/xf.log
timeout -k 10 300 python bench.py > gpurun_out/b_r1a.json 2> gpurun_out/b_r1a.err && \
CAPGEN_LNB_ROWS=2 timeout -k 10 300 python bench.py > gpurun_out/b_r2.json 2> gpurun_out/b_r2.err && \
timeout -k 10 300 python bench.py > gpurun_out/b_r1b.json 2> gpurun_out/b_r1b.err && \
for f in b_r1a b_r2 b_r1b; do python -c "import json,sys; d=json.loads(open('gpurun_out/$f.json').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['value'])"; done
