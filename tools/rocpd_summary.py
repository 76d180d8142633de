"""Per-kernel summary of a rocprofv3 run (its SQLite output, run_results.db): calls, mean and total
duration per kernel name, plus memory copies; optionally per call of a repeated workload (--per N).

  python tools/rocpd_summary.py gpurun_out/prof_x/run_results.db [--per 26] [--csv out.csv]
"""
import argparse
import csv
import sqlite3
import sys


def summary(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), avg(end - start), sum(end - start), min(end - start), "
                     "max(end - start) from kernels group by name order by 4 desc").fetchall()
    try:
        cp = c.execute("select count(*), sum(end - start) from memory_copies").fetchone()
    except sqlite3.Error:
        cp = (0, 0)
    return rows, cp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--per", type=int, default=0, help="divide totals by this many calls")
    ap.add_argument("--csv", default=None)
    a = ap.parse_args()
    rows, cp = summary(a.db)
    out = csv.writer(open(a.csv, "w", newline="") if a.csv else sys.stdout)
    out.writerow(["kernel", "calls", "avg_ns", "total_ns", "min_ns", "max_ns"] +
                 (["ns_per_workload_call"] if a.per else []))
    for name, n, avg, tot, mn, mx in rows:
        out.writerow([name, n, round(avg, 1), tot, mn, mx] + ([round(tot / a.per, 1)] if a.per else []))
    out.writerow(["(memory copies)", cp[0], "", cp[1] or 0, "", ""] + ([round((cp[1] or 0) / a.per, 1)] if a.per else []))


if __name__ == "__main__":
    main()
