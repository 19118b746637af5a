#!/bin/bash
# round 3: bench line, un-profiled stamp timeline of one step, persistent FFN pair vs plain pair,
# decode C4 (slab selection vs full-row), rocprofv3 kernel trace of a bench run
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
o=gpurun_out/r03
timeout -k 10 300 python -u tools/bench_generate.py > $o/gen.log 2>&1 || { tail -20 $o/gen.log; exit 4; }
grep '^{' $o/gen.log | cut -c1-200
CAPGEN_SLAB_DECODE=0 timeout -k 10 300 python -u tools/bench_generate.py > $o/gen_full.log 2>&1 || { tail -20 $o/gen_full.log; exit 5; }
grep '^{' $o/gen_full.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-batches > $o/trace.log 2>&1 || { tail -20 $o/trace.log; exit 6; }
d=$(dirname "$(find $o/trace -name run_kernel_trace.csv | head -1)")
cp "$d/run_kernel_stats.csv" $o/kernel_stats.csv
python tools/timeline.py "$d" --steps 10 > $o/timeline.txt
python tools/timeline.py "$d" --dominant >> $o/timeline.txt
head -12 $o/timeline.txt
rm -rf $o/trace
