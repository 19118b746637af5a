#!/bin/bash
# round 3: build the persisted tune table, run the ordering tests, one bench line
set -o pipefail
export CAPGEN_AUTOTUNE_LOG=1
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/tune_table.py --out gpurun_out/tune_gfx950.txt > gpurun_out/tune.log 2>&1 || exit 1
cp gpurun_out/tune_gfx950.txt image-caption_amd/capgen/tune_gfx950.txt
unset CAPGEN_AUTOTUNE_LOG
timeout -k 10 900 python -u -m pytest tests/test_gpu_hazard.py -x -v --timeout 300 --timeout-method thread > gpurun_out/hz.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-batches > gpurun_out/bench.log 2>&1 || exit 3
