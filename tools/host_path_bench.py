#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-memory batch path (north star: the path
starts in the client buffer and ends in the trie-resident value).  Times
lzf_host_compress_batch / lzf_host_decompress_batch on host arrays: staging
into pinned memory, hipMemcpyAsync H2D, kernels, D2H, copy-out -- for
DESIGN.md, never bench.py's `value`.
usage: host_path_bench.py [KIND N COUNT REPS]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gibson_amd  # noqa: E402


def main():
    kind, n, count, reps = (int(x, 0) for x in (sys.argv[1:5] if len(sys.argv) > 4
                                                 else ("1", "4096", "65536", "5")))
    syn = ctypes.CDLL(os.path.join(ROOT, "gibson_amd", "libgibson_synth.so"))
    syn.synth_fill.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                               ctypes.c_uint32, ctypes.c_void_p]
    arena = np.zeros(count * n, np.uint8)
    syn.synth_fill(kind, 0x5EED0002, 0, count, n, arena.ctypes.data)
    off = np.arange(count, dtype=np.uint64) * n
    ln = np.full(count, n, np.uint32)
    cap = np.full(count, n - 4, np.uint32)
    out = np.zeros_like(arena)
    olen = np.zeros(count, np.uint32)
    dec = np.zeros_like(arena)
    dlen = np.zeros(count, np.uint32)
    err = np.zeros(count, np.int32)
    tc, td = [], []
    for r in range(reps + 1):
        t0 = time.perf_counter()
        gibson_amd.host_compress_batch(arena, off, ln, out, off, cap, olen)
        t1 = time.perf_counter()
        ok = olen > 0
        gibson_amd.host_decompress_batch(out, off[ok], olen[ok], dec, off[ok], ln[ok], dlen, err)
        t2 = time.perf_counter()
        if r:
            tc.append(t1 - t0)
            td.append(t2 - t1)
    tc.sort()
    td.sort()
    c, d = tc[len(tc) // 2], td[len(td) // 2]
    good = bool((dlen[:ok.sum()] == n).all()) and np.array_equal(dec.reshape(count, n)[ok],
                                                                   arena.reshape(count, n)[ok])
    print(json.dumps({"path": "host memory -> pinned staging -> H2D -> kernel -> D2H -> host",
                      "kind": kind, "n": n, "count": count, "in_bytes": count * n,
                      "compress_GBps": round(count * n / c / 1e9, 3),
                      "decompress_GBps": round(count * n / d / 1e9, 3),
                      "roundtrip_GBps": round(count * n / (c + d) / 1e9, 3),
                      "roundtrip_ok": good, "kernels": gibson_amd.kernel_info()}))


if __name__ == "__main__":
    main()
