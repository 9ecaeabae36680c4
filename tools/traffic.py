#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-value HBM
traffic for bench.py's roofline.traffic.

gfx950 corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7):
FETCH_SIZE / WRITE_SIZE are in KiB; FETCH_SIZE reports half the bytes of a
wide coalesced streaming read, so it is doubled; WRITE_SIZE is taken as is.

A compress launch of the lane generation is two kernels (lzf_cand_*,
lzf_parse_lane); their per-dispatch traffic is summed into "lzf_compress",
as bench.py's compress time covers both.  Per-kernel figures are kept too.
usage: traffic.py PMC_DIR[,PMC_DIR...] WORKLOAD VALUES_PER_LAUNCH OUT_JSON
"""
import collections
import csv
import glob
import json
import sys

GROUPS = {
    "lzf_compress": ("compress_window", "compress_serial", "lzf_cand_", "lzf_parse_lane", "lzf_parse_rec"),
    "lzf_decompress": ("decompress",),
}


def group_of(name):
    for g, keys in GROUPS.items():
        if any(k in name for k in keys):
            return g
    return None


def main():
    d, workload, values, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    files = [f for dd in d.split(",") for f in glob.glob(dd + "/**/*counter_collection.csv", recursive=True)]
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0]
            if "lzf_" not in name or "synth" in name:
                continue
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {"workload": workload, "values_per_launch": values, "source": d,
           "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 per dispatch; a compress "
                         "launch sums its kernels", "kernels": {}, "per_kernel": {}}
    for k, c in acc.items():
        if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        # counters are per dispatch; a chunked launch dispatches a kernel several
        # times, so sum over the dispatches of one launch = mean * dispatches/launch
        fetch = sum(c["FETCH_SIZE"]) * 1024 * 2
        write = sum(c["WRITE_SIZE"]) * 1024
        res["per_kernel"][k] = {"read_bytes_per_value": fetch / values / max(1, launches(c)),
                                "write_bytes_per_value": write / values / max(1, launches(c))}
        g = group_of(k)
        if g:
            e = res["kernels"].setdefault(g, {"read_bytes_per_value": 0.0, "write_bytes_per_value": 0.0})
            e["read_bytes_per_value"] += res["per_kernel"][k]["read_bytes_per_value"]
            e["write_bytes_per_value"] += res["per_kernel"][k]["write_bytes_per_value"]
    for e in res["kernels"].values():
        e["bytes_per_value"] = e["read_bytes_per_value"] + e["write_bytes_per_value"]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


def launches(c):
    # the PMC passes run bench.py --steps 1 --warmup 0: one launch per kernel
    # group; TRAFFIC_LAUNCHES overrides for other invocations
    import os
    return int(os.environ.get("TRAFFIC_LAUNCHES", "1"))


if __name__ == "__main__":
    main()
