#!/bin/bash
# round 3: suite, bench line, un-profiled stamp timeline of one step, persistent FFN pair vs plain pair
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_check.sh tests bench || exit 1
timeout -k 10 300 python -u tools/stamp_timeline.py --out gpurun_out/stamps > gpurun_out/stamps.log 2>&1 || { tail -20 gpurun_out/stamps.log; exit 2; }
cat gpurun_out/stamps.log
timeout -k 10 300 python -u tools/persist_ffn.py > gpurun_out/persist.log 2>&1 || { tail -20 gpurun_out/persist.log; exit 3; }
cat gpurun_out/persist.log
timeout -k 10 300 python -u tools/bench_generate.py > gpurun_out/gen.log 2>&1 || { tail -20 gpurun_out/gen.log; exit 4; }
cat gpurun_out/gen.log
CAPGEN_SLAB_DECODE=0 timeout -k 10 300 python -u tools/bench_generate.py > gpurun_out/gen_full.log 2>&1 || { tail -20 gpurun_out/gen_full.log; exit 5; }
cat gpurun_out/gen_full.log
