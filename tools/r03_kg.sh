#!/bin/bash
# k-group GEMM variants: correctness, re-tune the table, per-shape sweep, bench with the new table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "k_groups or every_variant or k_tail" > gpurun_out/kg_tests.log 2>&1 || { tail -30 gpurun_out/kg_tests.log; exit 1; }
tail -2 gpurun_out/kg_tests.log
CAPGEN_AUTOTUNE_LOG=1 timeout -k 10 900 python -u tools/tune_table.py --out gpurun_out/tune_gfx950.txt > gpurun_out/tune.log 2>&1 || exit 2
cp gpurun_out/tune_gfx950.txt image-caption_amd/capgen/tune_gfx950.txt
timeout -k 10 900 python -u tools/gemm_splitk_sweep.py > gpurun_out/sksweep2.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host-batches > gpurun_out/bench_kg.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host-batches > gpurun_out/bench_kg2.log 2>&1 || exit 5
