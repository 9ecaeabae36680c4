#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter_collection CSVs per (kernel, counter)."""
import collections
import csv
import glob
import sys

tot = collections.defaultdict(float)
disp = collections.defaultdict(set)
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            short = k.split("(")[0][-60:]
            tot[(short, r["Counter_Name"])] += float(r["Counter_Value"])
            disp[short].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for (k, c), v in sorted(tot.items()):
    if "lzf" in k:
        print(f"{k:60s} {c:24s} {v:18.0f}  per-dispatch {v / max(1, len(disp[k])):16.0f}")
