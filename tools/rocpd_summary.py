#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (results.db) into the --stats kernel table and per-kernel PMC averages.

    python tools/rocpd_summary.py gpurun_out/<tag>/prof/bench_results.db > profiles/<name>_kernel_stats.csv
    python tools/rocpd_summary.py --pmc gpurun_out/<tag>/pmc_fetch/bench_results.db
"""
import argparse
import collections
import csv
import sqlite3
import sys


def kernel_stats(db):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
    for r in rows:
        w.writerow([r[0], r[1], f"{r[2]:.3f}", f"{r[3]:.3f}", f"{r[4]:.3f}"])


def pmc(db):
    c = sqlite3.connect(db)
    agg = collections.defaultdict(list)
    for k, n, v in c.execute("select kernel_name, counter_name, value from counters_collection"):
        agg[(k, n)].append(v)
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Counter", "Dispatches", "AveragePerDispatch"])
    for (k, n), v in sorted(agg.items()):
        w.writerow([k, n, len(v), f"{sum(v) / len(v):.3f}"])


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--pmc", action="store_true")
    a = ap.parse_args()
    (pmc if a.pmc else kernel_stats)(a.db)
