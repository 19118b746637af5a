"""Per-kernel stats (calls, total and average duration) from a rocprofv3 run's rocpd SQLite database
(the default output of `rocprofv3 --kernel-trace --stats` on this image), as the CSV of
`*_kernel_stats.csv`: python tools/rocpd_stats.py <results.db> [--top N]."""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=16)
    args = ap.parse_args()
    c = sqlite3.connect(args.db)
    print('"Name","Calls","TotalDurationNs","AverageNs"')
    q = "select name, count(*), sum(duration), avg(duration) from kernels group by name order by sum(duration) desc"
    for n, k, t, a in c.execute(q + " limit ?", (args.top,)):
        print('"%s",%d,%d,%.1f' % (n[:110], k, t, a))
    k, t = c.execute("select count(*), sum(duration) from kernels").fetchone()
    print("# all kernels: %d launches, %.3f ms" % (k, t / 1e6))


if __name__ == "__main__":
    main()
