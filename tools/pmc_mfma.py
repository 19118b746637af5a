"""MFMA utilisation per kernel class of one train step from a rocprofv3 PMC pass.

usage: python tools/pmc_mfma.py <pmc_dir> [out.json]

<pmc_dir> holds a `--pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace` run of bench.py.
Per MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES sums MFMA-busy cycles over every SIMD (one
v_mfma_f32_16x16x32_bf16 = 16 cycles = 16384 flop, i.e. 1024 flop per busy cycle); GRBM_GUI_ACTIVE
is summed over the 8 XCDs, so a dispatch lasts GRBM_GUI_ACTIVE / 8 shader cycles.  Utilisation =
MFMA busy / (1024 SIMDs x dispatch cycles) -- the fraction of the chip's dense MFMA issue the
kernel used while it ran (clock-independent, unlike TF/s against the 2.4 GHz peak).  Steps are
delimited by adam_prep_kernel as in tools/pmcsum.py; classes by tools/timeline.py's names.
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from timeline import short  # noqa: E402

N_SIMD = 1024


def main():
    f = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {sys.argv[1]}")
    by_disp = collections.defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(f[0])):
        d = int(r["Dispatch_Id"])
        by_disp[d][r["Counter_Name"]] = by_disp[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    disp = sorted(by_disp)
    marks = [i for i, d in enumerate(disp) if "adam_prep_kernel" in names[d]]
    n = min(5, len(marks) - 1)
    if n < 1:
        raise SystemExit("need at least two adam_prep_kernel markers")
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])  # launches, mfma busy, active cycles
    for d in disp[marks[-n - 1]:marks[-1]]:
        c = by_disp[d]
        a = agg[short(names[d])]
        a[0] += 1
        a[1] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        a[2] += c.get("GRBM_GUI_ACTIVE", 0.0) / 8
    tot_busy = sum(v[1] for v in agg.values())
    tot_cyc = sum(v[2] for v in agg.values())
    out = {"steps_averaged": n, "counters": "SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE (/8: per-XCD cycles)",
           "mfma_util_over_kernel_time": round(tot_busy / (N_SIMD * tot_cyc), 4) if tot_cyc else None,
           "mfma_gflop_per_step": round(tot_busy * 1024 / n / 1e9, 2),
           "per_kernel_class": {
               k: {"launches_per_step": v[0] / n, "mfma_util": round(v[1] / (N_SIMD * v[2]), 4) if v[2] else None,
                   "kernel_cycles_per_step": round(v[2] / n), "mfma_gflop_per_step": round(v[1] * 1024 / n / 1e9, 3)}
               for k, v in sorted(agg.items(), key=lambda kv: -kv[1][2]) if v[1] > 0 or v[2] > 0}}
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(s + "\n")


if __name__ == "__main__":
    main()
