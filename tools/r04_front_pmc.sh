#!/bin/bash
# round-4: why the fused self-attention front costs ~17 us regardless of rows / waves -- L2 hit / miss
# and fetched bytes of the microbench's kernels (tools/front_microbench.py), one PMC pass each
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04n
rm -rf $O && mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/hit -o run -- python3 tools/front_microbench.py > $O/hit.log 2>&1 || { tail -20 $O/hit.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- python3 tools/front_microbench.py > $O/fetch.log 2>&1 || { tail -20 $O/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv -d $O/sq -o run -- python3 tools/front_microbench.py > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 1; }
python - <<'PY'
import csv, glob, collections
O = "gpurun_out/r04n"
for tag in ("hit", "fetch", "sq"):
    f = glob.glob(f"{O}/{tag}/**/run_counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:60]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("==", tag)
    for k, c in acc.items():
        print(k, {n: round(sum(v) / len(v), 1) for n, v in c.items()})
PY
