"""Average every PMC counter per dispatch of the kernels whose name contains a pattern.

  python tools/pmc_kernel_avg.py <rocprofv3 output dir> [pattern=gemm_bf16_kernel] [--skip 1]

Reads the run's counter_collection.csv (rows: Dispatch_Id, Kernel_Name, Counter_Name, Counter_Value),
drops the first --skip dispatches of the pattern (warm-up), prints one JSON object: dispatches and the
mean of each counter.
"""
import argparse
import collections
import csv
import glob
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("pattern", nargs="?", default="gemm_bf16_kernel")
    ap.add_argument("--skip", type=int, default=1)
    a = ap.parse_args()
    f = glob.glob(f"{a.dir}/**/*counter_collection.csv", recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {a.dir}")
    by = collections.defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(f[0])):
        if a.pattern not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        by[d][r["Counter_Name"]] = by[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[d] = r["Kernel_Name"][:120]
    ids = sorted(by)[a.skip:]
    if not ids:
        raise SystemExit("no dispatches")
    keys = sorted({k for d in ids for k in by[d]})
    out = {"kernel": names[ids[0]], "dispatches": len(ids)}
    for k in keys:
        out[k] = sum(by[d].get(k, 0.0) for d in ids) / len(ids)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
