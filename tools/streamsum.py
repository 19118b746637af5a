"""Per-stream busy time and GPU idle per step from a rocprofv3 kernel trace (steps delimited by
adam_prep_kernel)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] + '/run_kernel_trace.csv')))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
marks = [i for i, r in enumerate(rows) if 'adam_prep_kernel' in r['Kernel_Name']]
n = min(10, len(marks) - 1)
sel = rows[marks[-n - 1]:marks[-1]]
wall = (int(rows[marks[-1]]['Start_Timestamp']) - int(sel[0]['Start_Timestamp'])) / n


def union(iv):
    iv = sorted(iv)
    tot, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + ce - cs


allv = [(int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in sel]
print(f"wall/step {wall / 1e3:.1f} us; GPU busy (any stream) {union(allv) / n / 1e3:.1f} us")
by = collections.defaultdict(list)
for r in sel:
    by[r.get('Stream_Id') or r['Queue_Id']].append(r)
for q, rs in sorted(by.items(), key=lambda kv: -len(kv[1])):
    iv = [(int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in rs]
    print(f"stream {q}: {len(rs) / n:5.1f} kernels/step, busy {union(iv) / n / 1e3:7.1f} us")
