#!/usr/bin/env python3
"""Per-phase cycle breakdown of the window64 compressor (diagnostic build).
usage: LZF_HIP_LIB=gibson_amd/liblzf_hip_stats.so python tools/cw_stats.py KIND N COUNT"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gibson_amd  # noqa: E402

PHASES = ["setup", "refill", "slots+masks", "lookup", "match+probe", "orbit+repair",
          "emit", "insert"]


def main():
    kind, n, count = (int(x, 0) for x in sys.argv[1:4])
    L = gibson_amd.lib()
    L.lzf_gpu_debug_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 32)()
    dev = "cuda"
    src = torch.empty(count * n, dtype=torch.uint8, device=dev)
    gibson_amd.synth_fill(kind, 0x5EED0002, 0, 1, count, n, src)
    off = torch.arange(count, dtype=torch.int64, device=dev) * n
    ln = torch.full((count,), n, dtype=torch.int32, device=dev)
    cap = torch.full((count,), n - 4, dtype=torch.int32, device=dev)
    out = torch.empty(count * n, dtype=torch.uint8, device=dev)
    ol = torch.zeros(count, dtype=torch.int32, device=dev)
    gibson_amd.compress_batch(src, off, ln, out, off, cap, ol, n)
    torch.cuda.synchronize()
    L.lzf_gpu_debug_stats(buf, 1)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    gibson_amd.compress_batch(src, off, ln, out, off, cap, ol, n)
    e1.record()
    torch.cuda.synchronize()
    L.lzf_gpu_debug_stats(buf, 1)
    st = list(buf)
    vals = max(1, st[5])
    w = max(1, st[0])
    print(f"kind {kind} n {n} count {count}: {e0.elapsed_time(e1):.2f} ms, "
          f"{count * n / e0.elapsed_time(e1) / 1e6:.2f} GB/s, ratio {float(ol.sum()) / (count * n):.4f}")
    print(f"windows/value {st[0] / vals:.1f}  repairs/value {st[1] / vals:.2f}  "
          f"unfinished-lookups/window {st[3] / w:.2f}  resolved-on-orbit/window {st[2] / w:.2f}  "
          f"orbit-matches/window {st[4] / w:.2f}  coop/window {st[6] / w:.2f}")
    tot = sum(st[8:8 + len(PHASES)])
    for i, name in enumerate(PHASES):
        c = st[8 + i]
        print(f"  {name:14s} {c / w:9.0f} cyc/window  {100.0 * c / max(1, tot):5.1f}%")


if __name__ == "__main__":
    main()
