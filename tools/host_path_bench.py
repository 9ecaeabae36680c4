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
import torch  # noqa: F401  (before the library: one HIP runtime in the process)

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
    seed = {0: 0x5EED0004, 1: 0x5EED0002, 2: 0x5EED0003, 3: 0x5EED0005}.get(kind, 0x5EED0002)
    syn.synth_fill(kind, seed, 0, count, n, arena.ctypes.data)
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
    parts = parts_of(arena, out, olen, n, count)
    cb = int(olen.astype(np.int64).sum())
    # the pipeline's overlap: the path's time against the sum of its parts
    # (bytes each part moves at its own measured rate)
    sum_c = count * n / parts["h2d_GBps"] + parts["compress_kernel_s"] * 1e9 + cb / parts["d2h_GBps"]
    sum_d = cb / parts["h2d_GBps"] + parts["decompress_kernel_s"] * 1e9 + count * n / parts["d2h_GBps"]
    print(json.dumps({"path": "host memory -> pinned staging -> H2D -> kernel -> D2H -> host",
                      "kind": kind, "seed": hex(seed), "n": n, "count": count, "in_bytes": count * n,
                      "compress_GBps": round(count * n / c / 1e9, 3),
                      "decompress_GBps": round(count * n / d / 1e9, 3),
                      "roundtrip_GBps": round(count * n / (c + d) / 1e9, 3),
                      "compress_s": round(c, 4), "decompress_s": round(d, 4),
                      "parts": parts,
                      "sum_of_parts_s": {"compress": round(sum_c / 1e9, 4), "decompress": round(sum_d / 1e9, 4)},
                      "overlap": {"compress": round(sum_c / 1e9 / c, 3), "decompress": round(sum_d / 1e9 / d, 3)},
                      "roundtrip_ok": good, "kernels": gibson_amd.kernel_info()}))


def parts_of(arena, out, olen, n, count):
    """the path's parts measured alone: pinned H2D and D2H of the arena, and
    the device-resident kernels on the same values"""
    import torch
    hp = torch.from_numpy(arena).pin_memory()
    dv = torch.empty(count * n, dtype=torch.uint8, device="cuda")
    t = []
    for r in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dv.copy_(hp, non_blocking=True)
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    h2d = count * n / sorted(t)[1] / 1e9
    t = []
    for r in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hp.copy_(dv, non_blocking=True)
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    d2h = count * n / sorted(t)[1] / 1e9
    off = torch.arange(count, dtype=torch.int64, device="cuda") * n
    ln = torch.full((count,), n, dtype=torch.int32, device="cuda")
    cap = torch.full((count,), n - 4, dtype=torch.int32, device="cuda")
    comp = torch.empty(count * n, dtype=torch.uint8, device="cuda")
    cl = torch.zeros(count, dtype=torch.int32, device="cuda")
    dec = torch.empty(count * n, dtype=torch.uint8, device="cuda")
    dl = torch.zeros(count, dtype=torch.int32, device="cuda")
    er = torch.zeros(count, dtype=torch.int32, device="cuda")
    tc, td = [], []
    for r in range(4):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        gibson_amd.compress_batch(dv, off, ln, comp, off, cap, cl, n)
        e1.record()
        ok = cl > 0
        gibson_amd.decompress_batch(comp, off, torch.where(ok, cl, torch.ones_like(cl)), dec, off,
                                    torch.where(ok, ln, torch.zeros_like(ln)), dl, er, n)
        e2.record()
        torch.cuda.synchronize()
        if r:
            tc.append(e0.elapsed_time(e1) / 1e3)
            td.append(e1.elapsed_time(e2) / 1e3)
    return {"h2d_GBps": round(h2d, 2), "d2h_GBps": round(d2h, 2),
            "compress_kernel_s": round(sorted(tc)[1], 5), "decompress_kernel_s": round(sorted(td)[1], 5)}


if __name__ == "__main__":
    main()
