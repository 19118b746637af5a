"""Timeline analysis of one train step from a rocprofv3 kernel trace (rocpd .db or CSV dir).

Usage: python tools/timeline.py <run_results.db | csv dir> [--list] [--steps K]

Steps are delimited by adam_prep_kernel (one per train step).  Prints, averaged over the
last K steps: wall per step, union of busy time (any kernel running), per-queue kernel
count / busy time, and the grouped kernel time; --list prints the kernels of the last
step in start order with their queue, duration and the gap before them on that queue.
"""
import collections
import csv
import os
import re
import sqlite3
import sys


def load(path):
    if path.endswith(".db"):
        db = sqlite3.connect(path)
        rows = db.execute("select name, queue_id, start, end, grid_x, workgroup_x from kernels").fetchall()
        return [dict(name=r[0], q=r[1], s=int(r[2]), e=int(r[3]), grid=r[4], wg=r[5]) for r in rows]
    rows = list(csv.DictReader(open(os.path.join(path, "run_kernel_trace.csv"))))
    return [dict(name=r["Kernel_Name"], q=int(r.get("Queue_Id", 0)), s=int(r["Start_Timestamp"]),
                 e=int(r["End_Timestamp"]), grid=int(r.get("Grid_Size_X", r.get("Grid_Size", 0))),
                 wg=int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 0)))) for r in rows]


def short(n):
    if "gemm_bf16_kernel" in n and "<" not in n:  # mangled: ...kernelI<TO>Lb<TA>ELb<TB>ELi<BM>E...
        m = re.search(r"gemm_bf16_kernelI(DF16b|f)Lb(\d)ELb(\d)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E", n)
        if m:
            to, ta, tb, bm, bn, wm, wn, st = m.groups()
            lay = {("0", "0"): "NT", ("0", "1"): "NN", ("1", "1"): "TN"}.get((ta, tb), ta + tb)
            return f"gemm {lay} {'bf16' if to == 'DF16b' else 'f32'} {bm}x{bn} w{int(wm) * int(wn)} s{st}"
    if "gemm_bf16_kernel" in n:
        return "gemm " + n[n.find("<"):n.find(">") + 1][:60]
    n = n.split("(")[0]
    return n.replace("void ", "").replace("capgen::", "")[-60:]


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def main():
    path = sys.argv[1]
    K = 5
    if "--steps" in sys.argv:
        K = int(sys.argv[sys.argv.index("--steps") + 1])
    rows = sorted(load(path), key=lambda r: r["s"])
    if "--dominant" in sys.argv:
        # bench.py's dominant_gemm(): the last 50 GEMM launches of the run (after 10 warm-ups)
        dom = [r for r in rows if "gemm_bf16_kernel" in r["name"]][-50:]
        avg = sum(r["e"] - r["s"] for r in dom) / len(dom) / 1e3
        print(f"dominant GEMM (bench.py dominant_gemm, last {len(dom)} launches): trace average {avg:.2f} us, "
              f"grid {dom[-1]['grid']}/{dom[-1]['wg']}, {short(dom[-1]['name'])}")
        return
    marks = [i for i, r in enumerate(rows) if "adam_prep_kernel" in r["name"]]
    K = min(K, len(marks) - 1)
    sel = rows[marks[-K - 1]:marks[-1]]
    t0, t1 = sel[0]["s"], rows[marks[-1]]["s"]
    print(f"wall per step {(t1 - t0) / 1e3 / K:.1f} us, kernels/step {len(sel) / K:.0f}, "
          f"busy(any) {union([(r['s'], r['e']) for r in sel]) / 1e3 / K:.1f} us, "
          f"sum of durations {sum(r['e'] - r['s'] for r in sel) / 1e3 / K:.1f} us")
    byq = collections.defaultdict(list)
    for r in sel:
        byq[r["q"]].append(r)
    for q, rs in sorted(byq.items()):
        busy = union([(r["s"], r["e"]) for r in rs])
        print(f"  queue {q}: {len(rs) / K:.0f} kernels, busy {busy / 1e3 / K:.1f} us, "
              f"sum {sum(r['e'] - r['s'] for r in rs) / 1e3 / K:.1f} us")
    agg = collections.defaultdict(lambda: [0, 0])
    for r in sel:
        k = short(r["name"])
        agg[k][0] += r["e"] - r["s"]
        agg[k][1] += 1
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0])[:25]:
        print(f"  {v[0] / 1e3 / K:8.1f} us  n={v[1] / K:5.1f}  avg {v[0] / v[1] / 1e3:6.2f}  {k}")
    if "--list" in sys.argv:
        last = rows[marks[-2]:marks[-1]]
        prev_end = {}
        base = last[0]["s"]
        for r in last:
            gap = r["s"] - prev_end.get(r["q"], r["s"])
            prev_end[r["q"]] = r["e"]
            print(f"{(r['s'] - base) / 1e3:8.1f} q{r['q']} {(r['e'] - r['s']) / 1e3:7.2f} us gap {gap / 1e3:6.2f}  "
                  f"grid {r['grid']:7d}/{r['wg']:4d}  {short(r['name'])}")


if __name__ == "__main__":
    main()
