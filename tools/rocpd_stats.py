#!/usr/bin/env python3
"""Kernel summary (name, calls, total/avg duration in us, %) from a rocprofv3
rocpd SQLite database, as the CSV --stats would write.
Usage: python tools/rocpd_stats.py RUN_results.db > stats.csv"""
import csv
import sqlite3
import sys


def main(path: str) -> None:
    c = sqlite3.connect(path)
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
    for name, calls, total, avg, pct in c.execute(
            "select name, total_calls, total_duration, average, percentage from top_kernels"):
        w.writerow([name, calls, f"{total:.3f}", f"{avg:.3f}", f"{pct:.4f}"])


if __name__ == "__main__":
    main(sys.argv[1])
