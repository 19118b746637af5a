#!/bin/bash
# round-4 check 5: decode attention query prefetch -- decode parity tests, then C4 generate x2
set -o pipefail
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "decode or c4 or beam or greedy or attention or fused" > $O/pytest_dec.log 2>&1 || { tail -40 $O/pytest_dec.log; exit 1; }
tail -2 $O/pytest_dec.log
for i in 1 2; do
timeout -k 10 300 python -u tools/bench_generate.py > $O/generate$i.json 2> $O/generate.err || { tail -20 $O/generate.err; exit 1; }
CAPGEN_DECODE_CROSS_MFMA=0 timeout -k 10 300 python -u tools/bench_generate.py --modes beam5 > $O/generate_valu$i.json 2> $O/generate.err || { tail -20 $O/generate.err; exit 1; }
cat $O/generate_valu$i.json
cat $O/generate$i.json
done
