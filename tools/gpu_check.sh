#!/bin/bash
# One GPU round trip: parity tests, the bench line, and a kernel-trace of a short bench run.
# Usage (on the GPU box, from the repo root): bash tools/gpu_check.sh [tests|bench|prof]...
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
steps=("$@")
[ ${#steps[@]} -eq 0 ] && steps=(tests bench prof)
for st in "${steps[@]}"; do
  case "$st" in
    tests)
      timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
      tail -2 gpurun_out/gpu_tests.log ;;
    bench)
      timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err \
        || { tail -20 gpurun_out/bench.err; exit 1; }
      cut -c1-330 gpurun_out/bench.json; echo ;;
    prof)
      rm -rf gpurun_out/prof
      timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
        python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-batches > gpurun_out/prof.log 2>&1 \
        || { tail -20 gpurun_out/prof.log; exit 1; }
      f=$(find gpurun_out/prof -name 'run_kernel_trace.csv' | head -1)
      mv "$(dirname "$f")"/run_* gpurun_out/prof/ 2>/dev/null
      python tools/timeline.py gpurun_out/prof | head -32 ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
