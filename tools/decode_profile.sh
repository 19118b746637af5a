#!/bin/bash
# C4 decode profile: bench_generate.py (beam-5 and greedy, B=256) plain, then each mode under
# rocprofv3 --kernel-trace (tools/lastcall.py on the last call) -> gpurun_out/<tag>/
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r02_decode}
out=gpurun_out/$tag
rm -rf "$out" && mkdir -p "$out"
timeout -k 10 200 python -u tools/bench_generate.py > "$out/generate.json" 2> "$out/generate.err" || { tail -20 "$out/generate.err"; exit 1; }
cat "$out/generate.json"
for m in beam5 greedy; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$out/trace_$m" -o run -- \
    python3 tools/bench_generate.py --reps 2 --modes $m > "$out/trace_$m.log" 2>&1 || { tail -20 "$out/trace_$m.log"; exit 1; }
  python tools/lastcall.py "$out/trace_$m" > "$out/lastcall_$m.txt"
  rm -rf "$out/trace_$m"
done
