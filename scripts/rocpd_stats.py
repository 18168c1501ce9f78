"""Kernel statistics (rocprofv3 --stats equivalent) from a rocprofv3 rocpd
database: name, calls, total / average / min / max duration (ns), share.
usage: python scripts/rocpd_stats.py <run_results.db> [out.csv]"""
import csv
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    rows = db.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), "
                      "max(end - start) from kernels group by name order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, n, s, a, lo, hi in rows:
        w.writerow([name, n, s, round(a, 1), round(100.0 * s / tot, 2), lo, hi])


if __name__ == "__main__":
    main()
