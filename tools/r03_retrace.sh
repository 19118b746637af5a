#!/bin/bash
# round 3 (after the LayerNorm-backward change): rocprofv3 kernel trace of a bench run + timeline
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03b
o=gpurun_out/r03b
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-batches > $o/trace.log 2>&1 || { tail -20 $o/trace.log; exit 6; }
grep '^{' $o/trace.log | tail -1 > $o/bench_traced.json
d=$(dirname "$(find $o/trace -name run_kernel_trace.csv | head -1)")
cp "$d/run_kernel_stats.csv" $o/kernel_stats.csv
python tools/timeline.py "$d" --steps 10 > $o/timeline.txt
python tools/timeline.py "$d" --dominant >> $o/timeline.txt
head -12 $o/timeline.txt
rm -rf $o/trace
