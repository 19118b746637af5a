#!/bin/bash
# round-4 check 16: branch-free K/V loads in the decode attention kernels -- parity subset, then the
# beam-5 decode kernel profile (per-kernel averages) and the decode bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04z
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "one_wave or attention_kernels or fused_attention_fronts or c4 or decode or beam or generate or greedy" > $O/pytest_ab.log 2>&1 || { tail -40 $O/pytest_ab.log; exit 1; }
tail -1 $O/pytest_ab.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/bench_generate.py --modes beam5 --reps 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name run_kernel_stats.csv | head -1)
grep -i "attn" $f | cut -d, -f1-4
for i in 1 2; do
timeout -k 10 300 python -u tools/bench_generate.py > $O/gen.$i.json 2> $O/gen.err || { tail -20 $O/gen.err; exit 1; }
cut -c1-150 $O/gen.$i.json
done
