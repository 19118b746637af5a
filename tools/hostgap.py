"""Split the critical-queue gaps of one train step into host-late vs device-side waits, from a
rocprofv3 --kernel-trace --hip-runtime-trace CSV directory (correlation ids link each kernel to the
API call that enqueued it).  Usage: python tools/hostgap.py <csv dir> [--list]"""
import csv
import os
import sys

d = sys.argv[1]
api = {}
for r in csv.DictReader(open(os.path.join(d, "run_hip_api_trace.csv"))):
    api[int(r["Correlation_Id"])] = (r["Function"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
ks = sorted((dict(name=r["Kernel_Name"], q=int(r["Queue_Id"]), s=int(r["Start_Timestamp"]),
                  e=int(r["End_Timestamp"]), c=int(r["Correlation_Id"]))
             for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv")))), key=lambda k: k["s"])
marks = [i for i, k in enumerate(ks) if "adam_prep_kernel" in k["name"]]
step = ks[marks[-3]:marks[-2]]
crit = max(set(k["q"] for k in step), key=lambda q: sum(1 for k in step if k["q"] == q))
prev = None
host_late = dev_wait = 0.0
rows = []
for k in step:
    if k["q"] != crit:
        continue
    fn, a0, a1 = api.get(k["c"], ("?", 0, 0))
    if prev is not None:
        gap = (k["s"] - prev["e"]) / 1e3
        late = max(0.0, min(gap, (a1 - prev["e"]) / 1e3))
        host_late += late
        dev_wait += gap - late
        rows.append((gap, late, k["name"][:70], fn, (k["s"] - step[0]["s"]) / 1e3))
    prev = k
print(f"critical queue {crit}: {len(rows) + 1} kernels, gaps {host_late + dev_wait:.1f} us = host-late "
      f"{host_late:.1f} us + device-side waits {dev_wait:.1f} us")
for gap, late, name, fn, t in sorted(rows, key=lambda r: -r[0])[:25]:
    print(f"  t={t:8.1f} gap {gap:7.2f} us (host-late {late:6.2f})  {fn:22s} {name}")
