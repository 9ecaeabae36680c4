#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-memory batch path (north star: the path
starts in the client buffer and ends in the trie-resident value).  Times
lzf_host_compress_batch / lzf_host_decompress_batch on host arrays: staging
into pinned memory, hipMemcpyAsync H2D, kernels, D2H, copy-out -- for
DESIGN.md, never bench.py's `value`.
usage: host_path_bench.py [KIND N COUNT REPS] [--register] [--devices LIST] [--arena-node N]
  --register  lzf_host_register the three arenas first (the GPU moves the
              values; no CPU packing)
  --devices   LZF_GPU_DEVICES for this process (e.g. 0,0 or all): value i to
              plan entry i mod G; the line reports each entry's spread"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def aligned(nbytes, node=None):
    """page-aligned zero bytes; with `node`, their pages bound to that NUMA
    node (mbind MPOL_BIND before the first touch)"""
    raw = np.zeros(nbytes + 8192, np.uint8)
    k = (-raw.ctypes.data) % 4096
    a = raw[k:k + nbytes]
    if node is not None:
        libc = ctypes.CDLL(None, use_errno=True)
        mask = ctypes.c_ulong(1 << node)
        # mbind(addr, len, MPOL_BIND = 2, nodemask, maxnode, MPOL_MF_MOVE = 2) -- syscall 237 on x86_64
        rc = libc.syscall(237, ctypes.c_void_p(a.ctypes.data), ctypes.c_ulong(nbytes), 2, ctypes.byref(mask),
                          ctypes.c_ulong(64), 2)
        if rc != 0:
            raise OSError(ctypes.get_errno(), f"mbind to node {node} refused")
    return a


def page_node(a):
    """the NUMA node holding the page at a's first byte (get_mempolicy
    MPOL_F_NODE | MPOL_F_ADDR, syscall 239), or -1"""
    libc = ctypes.CDLL(None, use_errno=True)
    mode = ctypes.c_int(-1)
    rc = libc.syscall(239, ctypes.byref(mode), None, ctypes.c_ulong(0), ctypes.c_void_p(a.ctypes.data), 3)
    return mode.value if rc == 0 else -1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pos", nargs="*", default=["1", "4096", "65536", "5"])
    ap.add_argument("--register", action="store_true")
    ap.add_argument("--devices", default=None)
    ap.add_argument("--arena-node", type=int, default=None,
                    help="bind the three host arenas' pages to this NUMA node (what a worker on the other "
                         "socket's GPU pays for an arena the caller allocated on its own node)")
    args = ap.parse_args()
    if args.devices:
        os.environ["LZF_GPU_DEVICES"] = args.devices      # read once, at the library's first host call
    import torch  # noqa: F401  (before the library: one HIP runtime in the process)
    import gibson_amd
    kind, n, count, reps = (int(x, 0) for x in (args.pos if len(args.pos) > 3 else ("1", "4096", "65536", "5")))
    syn = ctypes.CDLL(os.path.join(ROOT, "gibson_amd", "libgibson_synth.so"))
    syn.synth_fill.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                               ctypes.c_uint32, ctypes.c_void_p]
    arena = aligned(count * n, args.arena_node)
    seed = {0: 0x5EED0004, 1: 0x5EED0002, 2: 0x5EED0003, 3: 0x5EED0005}.get(kind, 0x5EED0002)
    syn.synth_fill(kind, seed, 0, count, n, arena.ctypes.data)
    off = np.arange(count, dtype=np.uint64) * n
    ln = np.full(count, n, np.uint32)
    cap = np.full(count, n - 4, np.uint32)
    out = aligned(count * n, args.arena_node)
    olen = np.zeros(count, np.uint32)
    dec = aligned(count * n, args.arena_node)
    out[::4096] = 0
    dec[::4096] = 0                                    # first touch: the pages land on the bound node
    dlen = np.zeros(count, np.uint32)
    err = np.zeros(count, np.int32)
    reg_s = None
    if args.register:
        t0 = time.perf_counter()
        for a in (arena, out, dec):
            gibson_amd.host_register(a)
        reg_s = time.perf_counter() - t0
    tc, td = [], []
    spread_c = spread_d = None
    for r in range(reps + 1):
        t0 = time.perf_counter()
        gibson_amd.host_compress_batch(arena, off, ln, out, off, cap, olen)
        t1 = time.perf_counter()
        spread_c = gibson_amd.host_last_spread()
        ok = olen > 0
        gibson_amd.host_decompress_batch(out, off[ok], olen[ok], dec, off[ok], ln[ok], dlen, err)
        t2 = time.perf_counter()
        spread_d = gibson_amd.host_last_spread()
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
    path = ("registered host arenas -> GPU gather / DMA runs -> kernel -> GPU scatter -> host" if args.register
            else "host memory -> pinned staging -> H2D -> kernel -> D2H -> host")
    plan = gibson_amd.device_plan()
    if args.register:
        for a in (arena, out, dec):
            gibson_amd.host_unregister(a)
    print(json.dumps({"path": path, "devices": plan, "register_s": reg_s,
                      "split": gibson_amd.host_split_policy(),
                      "arena_node": {"asked": args.arena_node, "first_page": [page_node(x) for x in (arena, out, dec)]},
                      "spread_last_rep": {"compress": [[v, round(ms, 2)] for v, ms in spread_c],
                                          "decompress": [[v, round(ms, 2)] for v, ms in spread_d]},
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
    import gibson_amd
    hp = torch.from_numpy(np.ascontiguousarray(arena)).pin_memory()
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
