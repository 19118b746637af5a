#!/bin/bash
# round-4 check 15: one-wave attention forward for Lq <= 16 (the beam's decode cross attention):
# bit-identity + torch parity, then decode A/B on CAPGEN_ATTN_WAVE
set -o pipefail
O=gpurun_out/r04y
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "one_wave or attention_kernels or fused_attention_fronts or c4 or decode or beam" > $O/pytest_ab.log 2>&1 || { tail -40 $O/pytest_ab.log; exit 1; }
tail -1 $O/pytest_ab.log
for i in 1 2; do
for w in 1 0; do
CAPGEN_ATTN_WAVE=$w timeout -k 10 300 python -u tools/bench_generate.py --modes beam5 > $O/gen$w.$i.json 2> $O/gen.err || { tail -20 $O/gen.err; exit 1; }
echo "wave $w $(cut -c1-160 $O/gen$w.$i.json)"
done
done
