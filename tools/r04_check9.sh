#!/bin/bash
# round-4 check 9: Adam writes the fronts' tiled weights itself -- full suite, bench, tile launches per step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s
rm -rf $O && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-batches > $O/bench$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench$i.json'));c=d['dominant_kernel']['classes_us_per_step'];print('bench', d['ms_per_step'], c)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-batches > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
grep -h "tile_weights\|adam_kernel" $(find $O/trace -name run_kernel_stats.csv) | cut -d, -f1-4
