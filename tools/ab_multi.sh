#!/bin/bash
# A/B several env settings on one box, R alternating rounds of a 100-step bench per setting:
#   bash tools/ab_multi.sh R "A=1 B=0" "A=1 B=1" ...   (prints ms/step per run, then the means)
set -o pipefail
mkdir -p gpurun_out
R=$1; shift
declare -A sum
for round in $(seq 1 "$R"); do
  for spec in "$@"; do
    env $spec timeout -k 10 120 python -u bench.py --steps 100 --no-cpu-baseline --no-host-batches > gpurun_out/ab.json 2> gpurun_out/ab.err \
      || { tail -20 gpurun_out/ab.err; exit 1; }
    ms=$(python3 -c "import json; print(json.load(open('gpurun_out/ab.json'))['ms_per_step'])")
    echo "[$spec] $ms"
    sum[$spec]=$(python3 -c "print(${sum[$spec]:-0} + $ms)")
  done
done
for spec in "$@"; do python3 -c "print('mean [$spec]', round(${sum[$spec]} / $R, 4))"; done
