"""Per-shape kernel durations from a rocprofv3 kernel trace of tools/gemm_time.py: the run issues
1 + reps launches of the library GEMM per shape in order; this groups the gemm_bf16 dispatches
in that order and prints each group's mean duration (the first launch of each dropped).

  python tools/trace_groups.py <rocprofv3 output dir> [--reps 200] [--pattern gemm_bf16]
"""
import argparse
import csv
import glob


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--pattern", default="gemm_bf16")
    a = ap.parse_args()
    f = glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if a.pattern in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    g = a.reps + 1
    for i in range(0, len(rows), g):
        grp = rows[i + 1:i + g]
        if not grp:
            break
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in grp]
        print(f"group {i // g}: {len(d)} launches, mean {sum(d) / len(d):7.2f} us, min {min(d):7.2f}  "
              f"{grp[0]['Kernel_Name'][:90]}")


if __name__ == "__main__":
    main()
