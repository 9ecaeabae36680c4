#!/usr/bin/env python3
"""Cycles per phase of the window parse (lzf_wparse.hip built with
-DWP_TIMING: tools/build_variant.sh wpt -DWP_TIMING with SRC=lzf_wparse.hip).
usage: LZF_HIP_LIB=gibson_amd/liblzf_hip_wpt.so wp_timing.py KIND SEED N COUNT"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["LZF_GPU_KERNEL"] = "wtab"
import torch  # noqa: E402

import gibson_amd  # noqa: E402

kind, seed, n, count = int(sys.argv[1]), int(sys.argv[2], 0), int(sys.argv[3]), int(sys.argv[4])
L = gibson_amd.lib()
fn = L.lzf_gpu_debug_wp
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
src = torch.empty(count * n, dtype=torch.uint8, device="cuda")
gibson_amd.synth_fill(kind, seed, 0, 1, count, n, src)
off = torch.arange(count, dtype=torch.int64, device="cuda") * n
ln = torch.full((count,), n, dtype=torch.int32, device="cuda")
cap = torch.full((count,), n - 4, dtype=torch.int32, device="cuda")
out = torch.empty(count * n, dtype=torch.uint8, device="cuda")
olen = torch.zeros(count, dtype=torch.int32, device="cuda")
gibson_amd.compress_batch(src, off, ln, out, off, cap, olen, n)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 16)()
fn(buf, 1)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
gibson_amd.compress_batch(src, off, ln, out, off, cap, olen, n)
e1.record()
torch.cuda.synchronize()
fn(buf, 0)
t = list(buf)
win = max(t[8], 1)
names = ["links", "ring", "loads+len", "walk", "extend", "emit", "ring upd"]
print(f"compress {e0.elapsed_time(e1):.2f} ms; windows {t[8]} active {t[9]} stops/active {t[10]/max(t[9],1):.2f} "
      f"ext/active {t[11]/max(t[9],1):.3f} doubling rounds/window {t[12]/win:.2f}")
tot = sum(t[:7])
for i, nm in enumerate(names):
    print(f"  {nm:10s} {t[i]/win:9.1f} cycles/window  {100*t[i]/max(tot,1):5.1f}%")
