#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (kernel stats) as CSV + text.

usage: tools/rocpd_summary.py <results.db> <out_prefix>
Writes <out_prefix>_kernel_stats.csv (name, calls, total_us, avg_us, min_us,
max_us, pct) and prints the same table.
"""
import csv
import sqlite3
import sys


def main(db, prefix):
    c = sqlite3.connect(db)
    rows = list(c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
        "from kernels group by name order by sum(duration) desc"))
    tot = sum(r[2] for r in rows) or 1
    with open(prefix + "_kernel_stats.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["name", "calls", "total_us", "avg_us", "min_us", "max_us", "pct"])
        for name, n, s, a, mn, mx in rows:
            w.writerow([name, n, "%.3f" % (s / 1e3), "%.3f" % (a / 1e3), "%.3f" % (mn / 1e3),
                        "%.3f" % (mx / 1e3), "%.2f" % (100.0 * s / tot)])
    for name, n, s, a, mn, mx in rows:
        print("%7d calls %10.1f us total %8.3f us avg %6.2f%%  %s" % (n, s / 1e3, a / 1e3, 100.0 * s / tot, name))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
