#!/bin/bash
# GPU-box check of the current tree (run from the repo root through gpurun):
#   bash tools/gpu_check.sh <tag> [suite] [smoke] [bench] [ab:<arm>;<arm>...]
# writes gpurun_out/<tag>/: suite.log (pytest -m gpu), smoke.log, bench.json.  Each step has its own
# time limit; a GPU fault, abort, segfault or time-out (rc 124 / 134 / 137 / 139) ends the script
# there; an ordinary test failure (rc 1) is reported and the next step still runs.
set -o pipefail
tag=${1:?tag}
shift
out=gpurun_out/$tag
mkdir -p "$out"
fatal() { case "$1" in 124|134|137|139) return 0 ;; *) return 1 ;; esac; }
for step in "$@"; do
  case "$step" in
    suite)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/suite.log" 2>&1
      rc=$?; tail -3 "$out/suite.log"; echo "[suite rc $rc]"; fatal $rc && exit $rc ;;
    smoke)
      timeout -k 10 200 python -u -c 'import __graft_entry__ as g; g.smoke()' > "$out/smoke.log" 2>&1
      rc=$?; tail -2 "$out/smoke.log"; echo "[smoke rc $rc]"; fatal $rc && exit $rc ;;
    bench)
      timeout -k 10 300 python -u bench.py > "$out/bench.json" 2> "$out/bench.err"
      rc=$?; cut -c1-600 "$out/bench.json"; echo "[bench rc $rc]"; fatal $rc && exit $rc ;;
    ab:*)
      arms=${step#ab:}
      args=()
      IFS=';' read -ra A <<< "$arms"
      for a in "${A[@]}"; do args+=(--arm "$a"); done
      timeout -k 10 600 python -u tools/ab.py --rounds 3 --out "$out/ab.jsonl" "${args[@]}" > "$out/ab.log" 2>&1
      rc=$?; tail -6 "$out/ab.log"; echo "[ab rc $rc]"; fatal $rc && exit $rc ;;
  esac
done
exit 0
