#!/bin/bash
# Per-kernel average durations (by name and grid) under each env spec, from a short rocprofv3
# kernel trace of bench.py; pattern selects kernels: bash tools/kavg.sh PATTERN "ENV=a" "ENV=b" ...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
pat=$1; shift
i=0
for spec in "$@"; do
  i=$((i + 1)); d=gpurun_out/kavg$i; rm -rf "$d"
  env $spec timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-batches > "$d.log" 2>&1 || { tail -20 "$d.log"; exit 1; }
  f=$(find "$d" -name run_kernel_trace.csv | head -1)
  python3 - "$f" "$pat" "$spec" <<'PY'
import csv, re, sys, collections
f, pat, spec = sys.argv[1:4]
rows = list(csv.DictReader(open(f)))
rows = rows[len(rows) // 2:]  # the second half: tuned, steady state
acc = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if re.search(pat, n):
        acc[(n[:60], r.get("Grid_Size_X", r.get("Grid_Size")))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (n, g), v in sorted(acc.items()):
    print(f"[{spec}] {n:60s} grid {g:>8s} n={len(v):4d} avg {sum(v)/len(v):7.2f} us")
PY
  rm -rf "$d"
done
