#!/bin/bash
# round-4 check 2: -m gpu suite, bench, C4 decode bench, persistent-FFN small diagnostic
set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-batches > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json; python -c "import json;d=json.load(open('$O/bench.json'));print(d['dominant_kernel'])"
timeout -k 10 300 python -u tools/bench_generate.py > $O/generate.json 2> $O/generate.err || { tail -20 $O/generate.err; exit 1; }
cat $O/generate.json
timeout -k 10 120 python -u tools/persist_ffn.py --small > $O/persist_small.log 2>&1 || { cat $O/persist_small.log; exit 1; }
cat $O/persist_small.log
