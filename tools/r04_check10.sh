#!/bin/bash
# round-4 check 10: decode GEMMs re-tuned with deeper split-K allowed (>= 2 k-tiles per slice)
set -o pipefail
O=gpurun_out/r04t
mkdir -p $O
T=image-caption_amd/capgen/tune_gfx950.txt
CAPGEN_AUTOTUNE_LOG=1 timeout -k 10 600 python -u tools/retune_decode.py $T $O/tune_new.txt > $O/retune.log 2>&1 || { tail -20 $O/retune.log; exit 1; }
grep "capgen gemm\|live" $O/retune.log | grep -v "tune table" | tail -12
for i in 1 2; do
timeout -k 10 300 python -u tools/bench_generate.py > $O/gen_old$i.json 2> $O/gen.err || { tail -20 $O/gen.err; exit 1; }
CAPGEN_TUNE_TABLE=$PWD/$O/tune_new.txt timeout -k 10 300 python -u tools/bench_generate.py > $O/gen_new$i.json 2> $O/gen.err || { tail -20 $O/gen.err; exit 1; }
echo old; cat $O/gen_old$i.json; echo new; cat $O/gen_new$i.json
done
