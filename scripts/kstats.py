"""Kernel statistics (name, calls, total / average / min / max duration) from
a rocprofv3 results database (the default --output-format of rocprofv3 on
this image), written as CSV like rocprofv3's kernel_stats.csv.
usage: python scripts/kstats.py <run_results.db> [out.csv]"""
import csv
import sqlite3
import sys


def stats(db_path):
    db = sqlite3.connect(db_path)
    rows = db.execute(
        "select name, count(*), sum(end - start), avg(end - start), min(end - start), "
        "max(end - start) from kernels group by name order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    return [(n, c, t, a, mn, mx, 100.0 * t / total) for n, c, t, a, mn, mx in rows]


def main():
    rows = stats(sys.argv[1])
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
    for r in rows:
        w.writerow([r[0], r[1], r[2], round(r[3], 1), r[4], r[5], round(r[6], 2)])


if __name__ == "__main__":
    main()
