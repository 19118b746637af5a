#!/bin/bash
# Per-kernel average durations of a short bench run under an env setting:
#   bash tools/kstat.sh <tag> [VAR=value ...]   -> gpurun_out/kstat_<tag>.csv (rocprofv3 --stats)
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
rm -rf gpurun_out/ks_$tag
env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_$tag -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-batches > gpurun_out/ks_$tag.log 2>&1 || { tail -5 gpurun_out/ks_$tag.log; exit 1; }
f=$(find gpurun_out/ks_$tag -name run_kernel_stats.csv | head -1)
cp "$f" gpurun_out/kstat_$tag.csv
rm -rf gpurun_out/ks_$tag
