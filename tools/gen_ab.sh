#!/bin/bash
# Alternating C4 generate runs of two libraries (decode A/B):  bash tools/gen_ab.sh <tag> <lib_a> <lib_b> [rounds]
set -o pipefail
tag=${1:?tag}; a=${2:?lib a}; b=${3:?lib b}; n=${4:-3}
out=gpurun_out/$tag; mkdir -p "$out"
for r in $(seq 1 "$n"); do
  for arm in a b; do
    lib=$a; [ $arm = b ] && lib=$b
    CAPGEN_LIB_PATH=$lib timeout -k 10 120 python -u tools/bench_generate.py --reps 5 > "$out/gen_${arm}_$r.jsonl" 2>/dev/null || { echo "rc $? ($arm round $r)"; exit 1; }
    echo "$arm round $r: $(python -c "import json,sys;print(' '.join(f\"{json.loads(l)['metric'].split()[1]} {json.loads(l)['ms_per_batch']}\" for l in open('$out/gen_${arm}_$r.jsonl') if l.startswith('{')))")"
  done
done
