#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-value HBM
traffic for bench.py's roofline.traffic.

gfx950 corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7):
FETCH_SIZE / WRITE_SIZE are in KiB; FETCH_SIZE reports half the bytes of a
wide coalesced streaming read, so it is doubled; WRITE_SIZE is taken as is.
usage: traffic.py PMC_DIR[,PMC_DIR...] WORKLOAD VALUES_PER_LAUNCH OUT_JSON
"""
import collections
import csv
import glob
import json
import sys


def main():
    d, workload, values, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    files = [f for dd in d.split(",") for f in glob.glob(dd + "/**/*counter_collection.csv", recursive=True)]
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0]
            if "lzf_" not in name:
                continue
            key = "lzf_compress" if "compress_window" in name or "compress_serial" in name else \
                  "lzf_decompress" if "decompress" in name else name
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {"workload": workload, "values_per_launch": values, "source": d,
           "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 per dispatch", "kernels": {}}
    for k, c in acc.items():
        if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        fetch = sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"]) * 1024 * 2
        write = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"]) * 1024
        res["kernels"][k] = {"read_bytes_per_value": fetch / values,
                             "write_bytes_per_value": write / values,
                             "bytes_per_value": (fetch + write) / values}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
