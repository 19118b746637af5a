#!/bin/bash
# round-3 final check: -m gpu suite, smoke(), bench line, decode bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final
o=gpurun_out/final
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -1 $o/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 2; }
tail -1 $o/smoke.log
timeout -k 10 300 python -u bench.py > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 3; }
cut -c1-260 $o/bench.json
timeout -k 10 300 python -u tools/bench_generate.py > $o/gen.log 2>&1 || { tail -20 $o/gen.log; exit 4; }
grep '^{' $o/gen.log | cut -c1-200
