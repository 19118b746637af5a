#!/bin/bash
# round-4 check on the GPU box: -m gpu suite (+ the C2 gradient error table), bench, then the
# persistent-FFN experiment (bounded: every wait in the kernel gives up after 2 s)
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
export CAPGEN_REPORT_DIR=$O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-batches > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 120 python -u tools/persist_ffn.py --small > $O/persist_small.log 2>&1 || { cat $O/persist_small.log; exit 1; }
cat $O/persist_small.log
timeout -k 10 300 python -u tools/persist_ffn.py --reps 20 > $O/persist.log 2>&1 || { tail -20 $O/persist.log; exit 1; }
cat $O/persist.log
