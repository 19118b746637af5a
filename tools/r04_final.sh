#!/bin/bash
# round-4 final check: -m gpu suite, smoke(), bench line (default args), decode bench
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04final
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -1 $o/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 2; }
tail -1 $o/smoke.log
timeout -k 10 400 python -u bench.py > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 3; }
cut -c1-300 $o/bench.json
timeout -k 10 300 python -u tools/bench_generate.py > $o/gen.json 2> $o/gen.err || { tail -20 $o/gen.err; exit 4; }
cat $o/gen.json
