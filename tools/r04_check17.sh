#!/bin/bash
# round-4 check 17: the one-wave attention forward (loads of rows past Lk skipped) -- full -m gpu
# suite, then the beam-5 decode kernel profile and two decode bench runs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04aa
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/bench_generate.py --modes beam5 --reps 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name run_kernel_stats.csv | head -1)
cp $f $O/decode_kernel_stats.csv
grep -i "attn" $f | cut -d, -f1-4
for i in 1 2; do
for w in 1 0; do
CAPGEN_ATTN_WAVE=$w timeout -k 10 300 python -u tools/bench_generate.py --modes beam5 > $O/gen$w.$i.json 2> $O/gen.err || { tail -20 $O/gen.err; exit 1; }
echo "wave $w $(cut -c1-150 $O/gen$w.$i.json)"
done
done
