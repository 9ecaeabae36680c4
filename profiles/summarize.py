#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats output (SQLite .db or
kernel_stats.csv) into the compact table committed under profiles/.
usage: summarize.py <rocprof output dir> [label]"""
import csv
import glob
import os
import sqlite3
import sys


def rows(d):
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    if dbs:
        c = sqlite3.connect(dbs[0])
        for name, calls, total, avg, pct in c.execute(
                "select name, total_calls, total_duration, average, percentage from top_kernels"):
            yield name, int(calls), float(total), float(avg), float(pct)   # durations in us
        return
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            yield (r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                   float(r["AverageNs"]) / 1e3, float(r["Percentage"]))


def main():
    d = sys.argv[1]
    label = sys.argv[2] if len(sys.argv) > 2 else d
    print(f"# rocprofv3 --kernel-trace --stats summary: {label}")
    print(f"{'calls':>6} {'total_ms':>11} {'avg_us':>12} {'pct':>6}  kernel")
    for name, calls, total, avg, pct in rows(d):
        short = name if len(name) < 110 else name[:107] + "..."
        print(f"{calls:6d} {total / 1e3:11.3f} {avg:12.1f} {pct:6.2f}  {short}")


if __name__ == "__main__":
    main()
