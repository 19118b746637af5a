#!/bin/bash
# round-4: ce_finish + loss_finalize (the merged form was reverted) -- CE tests, kernel time, step gap
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04q
rm -rf $O && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "fused_classifier_ce or focal or loss_path or c2_full_size or train_step or bucketed" > $O/pytest_ce.log 2>&1 || { tail -40 $O/pytest_ce.log; exit 1; }
tail -1 $O/pytest_ce.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-batches > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
grep -h "ce_finish\|loss_finalize" $(find $O/trace -name run_kernel_stats.csv) | cut -d, -f1-5
timeout -k 10 300 python -u tools/stamp_timeline.py --out $O/stamps > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
tail -2 $O/stamps.log
python -c "
import json;d=json.load(open('$O/stamps/summary.json'))
for g in d['reps'][0]['largest_gaps'][:3]: print(g)
"
