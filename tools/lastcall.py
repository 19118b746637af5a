"""Kernel time of the LAST call in a rocprofv3 kernel trace whose calls each start with one
pack_kernel launch (encode_only): per-kernel-class totals, launches and the call's wall span.
usage: python tools/lastcall.py <trace csv dir> [--top K]"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from timeline import short  # noqa: E402


def main():
    d = sys.argv[1]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 25
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "pack_kernel" in r["Kernel_Name"]]
    last = rows[starts[-1]:]
    t0, t1 = int(last[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in last)
    agg = collections.defaultdict(lambda: [0, 0])
    for r in last:
        a = agg[short(r["Kernel_Name"])]
        a[0] += 1
        a[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    busy = sum(v[1] for v in agg.values())
    print(f"last call: wall {(t1 - t0) / 1e6:.3f} ms, {len(last)} kernels, kernel time {busy / 1e6:.3f} ms")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{v[1] / 1e6:8.3f} ms  n={v[0]:5d}  avg {v[1] / v[0] / 1e3:8.2f} us  {k}")


if __name__ == "__main__":
    main()
