"""HBM bytes per train step from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

usage: python tools/pmcsum.py <fetch_dir> <write_dir> [out.json]

Each dir holds a `--pmc <counter> --kernel-trace` run of `bench.py --no-graph` (counter
collection serialises dispatches, so the eager path is profiled; it launches the same kernels
as the graph replay).  Steps are delimited by the one adam_prep_kernel launch per step; the
last few complete steps are averaged.  Per MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE
(kB) is doubled on gfx950 for wide streaming reads; WRITE_SIZE (kB) is taken as is.
"""
import collections
import csv
import glob
import json
import os
import sys


def per_kernel(d, counter):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    rows = [r for r in csv.DictReader(open(f[0])) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def step_slices(rows, nmax=5):
    marks = [i for i, r in enumerate(rows) if "adam_prep_kernel" in r["Kernel_Name"]]
    n = min(nmax, len(marks) - 1)
    if n < 1:
        raise SystemExit("need at least two adam_prep_kernel markers")
    return rows[marks[-n - 1]:marks[-1]], n


def short(name):
    return "gemm_bf16" if "gemm_bf16_kernel" in name else name.split("(")[0].split("<")[0][-40:]


def main():
    fetch, nf = step_slices(per_kernel(sys.argv[1], "FETCH_SIZE"))
    write, nw = step_slices(per_kernel(sys.argv[2], "WRITE_SIZE"))
    agg = collections.defaultdict(lambda: [0.0, 0.0])
    for r in fetch:
        agg[short(r["Kernel_Name"])][0] += 2.0 * float(r["Counter_Value"]) * 1024 / nf
    for r in write:
        agg[short(r["Kernel_Name"])][1] += float(r["Counter_Value"]) * 1024 / nw
    rd = sum(v[0] for v in agg.values())
    wr = sum(v[1] for v in agg.values())
    # the commit the profiled tree was (tools/round_profile.sh passes it: the GPU box has no .git), so a
    # bench line quoting this file shows which code its traffic belongs to
    out = {"commit": os.environ.get("CAPGEN_COMMIT", "unknown"),
           "hbm_bytes_per_step": round(rd + wr), "read_bytes_per_step": round(rd), "write_bytes_per_step": round(wr),
           "steps_averaged": [nf, nw], "correction": "FETCH_SIZE x2 (gfx950 wide-read), kB x1024",
           "per_kernel_class": {k: {"read": round(v[0]), "write": round(v[1])}
                                for k, v in sorted(agg.items(), key=lambda kv: -(kv[1][0] + kv[1][1]))}}
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s + "\n")


if __name__ == "__main__":
    main()
