#!/usr/bin/env python3
"""Timeline of kernels and copies from a rocprofv3 --kernel-trace
--memory-copy-trace CSV pair: one line per event longer than MIN_MS, times in
ms from the start of the window.  usage: trace_timeline.py DIR PREFIX [FROM_MS SPAN_MS MIN_MS]"""
import csv
import os
import sys


def main():
    d, pre = sys.argv[1], sys.argv[2]
    t_from, span, min_ms = (float(x) for x in (sys.argv[3:6] if len(sys.argv) > 5 else ("0", "1e9", "0.3")))
    ev = []
    for r in csv.DictReader(open(os.path.join(d, pre + "_kernel_trace.csv"))):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "kernel", r["Kernel_Name"].split("(")[0],
                   r["Stream_Id"]))
    mc = os.path.join(d, pre + "_memory_copy_trace.csv")
    if os.path.exists(mc):
        for r in csv.DictReader(open(mc)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy",
                       r["Direction"].replace("MEMORY_COPY_", ""), r["Stream_Id"]))
    ev.sort()
    t0 = ev[0][0] + t_from * 1e6
    for s, e, kind, name, stream in ev:
        if s < t0 or s > t0 + span * 1e6 or (e - s) < min_ms * 1e6:
            continue
        print(f"{(s - t0) / 1e6:10.2f} {(e - t0) / 1e6:10.2f} {(e - s) / 1e6:8.2f}  stream {stream:>3}  {kind:6s} {name}")


if __name__ == "__main__":
    main()
