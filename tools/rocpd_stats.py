#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 results database (ROCm 7's default
output, `<name>_results.db`: the `top_kernels` view), as CSV.

    python tools/rocpd_stats.py gpurun_out/r5h/prof2048/p_results.db > stats.csv
"""
import csv
import sqlite3
import sys


def main():
    if len(sys.argv) != 2:
        print(__doc__, file=sys.stderr)
        return 2
    db = sqlite3.connect(sys.argv[1])
    w = csv.writer(sys.stdout)
    w.writerow(["name", "calls", "total_us", "average_us", "percent"])
    for name, calls, tot, avg, pct in db.execute(
            "select name, total_calls, total_duration, average, percentage from top_kernels"):
        w.writerow([name, calls, round(float(tot), 3), round(float(avg), 3), round(float(pct), 3)])
    return 0


if __name__ == "__main__":
    sys.exit(main())
