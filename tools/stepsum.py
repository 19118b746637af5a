"""Per-step kernel-time breakdown from a rocprofv3 --kernel-trace CSV (steps delimited by Adam)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] + '/run_kernel_trace.csv')))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
marks = [i for i, r in enumerate(rows) if 'adam_prep_kernel' in r['Kernel_Name']]
nsteps = min(10, len(marks) - 1)
sel = rows[marks[-nsteps - 1]:marks[-1]]
t0 = int(sel[0]['Start_Timestamp'])
t1 = max(int(r['End_Timestamp']) for r in sel)
print(f'wall per step {(t1 - t0) / 1e6 / nsteps:.3f} ms, kernels/step {len(sel) / nsteps:.0f}')
agg = collections.defaultdict(lambda: [0, 0])
for r in sel:
    n = r['Kernel_Name']
    key = 'gemm' if 'gemm_bf16_kernel' in n else n.split('(')[0].split('<')[0][-40:]
    agg[key][0] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    agg[key][1] += 1
print(f'sum of kernel durations per step {sum(v[0] for v in agg.values()) / 1e6 / nsteps:.3f} ms')
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0])[:int(sys.argv[2]) if len(sys.argv) > 2 else 14]:
    print(f"{v[0] / 1e6 / nsteps:7.3f} ms  n={v[1] / nsteps:5.1f}  {k}")
