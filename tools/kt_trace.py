#!/usr/bin/env python3
"""Per-step busy cycles of every wave of lzf_cand_table_kernel (diagnostic
build gibson_amd/liblzf_hip_ktlite.so, -DKT_TIMING -DKT_LITE): for the first
64 workgroups, each wave's cycles from the step's start to the barrier, one
value's steps.  Prints the kernel time (the build runs at the product's
speed) and how the step's critical path splits: the table wave against the
slowest of the 15 workers.   usage: kt_trace.py KIND N COUNT"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("LZF_HIP_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gibson_amd",
                                                  "liblzf_hip_ktlite.so"))
os.environ.setdefault("LZF_GPU_TABLE_STAGE", "1")
os.environ.setdefault("LZF_GPU_LANE_MIN", "0")
import torch  # noqa: E402

import gibson_amd  # noqa: E402

SEEDS = {0: 0x5EED0004, 1: 0x5EED0002, 2: 0x5EED0003, 3: 0x5EED0005}
kind, n, count = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
L = gibson_amd.lib()
L.lzf_gpu_debug_kt_trace.argtypes = [ctypes.c_void_p]
src = torch.empty(count * n, dtype=torch.uint8, device="cuda")
gibson_amd.synth_fill(kind, SEEDS.get(kind, 0x5EED0002), 0, 1, count, n, src)
off = torch.arange(count, dtype=torch.int64, device="cuda") * n
ln = torch.full((count,), n, dtype=torch.int32, device="cuda")
cap = torch.full((count,), n - 4, dtype=torch.int32, device="cuda")
out = torch.empty(count * n, dtype=torch.uint8, device="cuda")
olen = torch.zeros(count, dtype=torch.int32, device="cuda")
gibson_amd.compress_batch(src, off, ln, out, off, cap, olen, n)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
gibson_amd.compress_batch(src, off, ln, out, off, cap, olen, n)
e1.record()
torch.cuda.synchronize()
tr = np.zeros(64 * 4096 * 16, np.uint32)
assert L.lzf_gpu_debug_kt_trace(tr.ctypes.data) == 0
tr = tr.reshape(64, 4096, 16)
steps = tr[:, :, 0] > 0
tb = tr[:, :, 0][steps].astype(np.float64)
wk = tr[:, :, 1:16][steps].astype(np.float64)
wmax, wmean = wk.max(axis=1), wk.mean(axis=1)
crit = np.maximum(tb, wmax)
print(f"kernel {e0.elapsed_time(e1):.2f} ms (cand alone, {count} x {n} B), {int(steps.sum())} sampled steps")
print(f"  table wave busy        mean {tb.mean():8.0f}  median {np.median(tb):8.0f}")
print(f"  worker busy            mean {wmean.mean():8.0f}  (per step, over the 15 workers)")
print(f"  slowest worker busy    mean {wmax.mean():8.0f}  median {np.median(wmax):8.0f}  p90 {np.percentile(wmax, 90):8.0f}")
print(f"  max(table, workers)    mean {crit.mean():8.0f}")
print(f"  steps where the table wave is the last to arrive: {100.0 * (tb >= wmax).mean():.1f} %")
print(f"  slowest worker's excess over the mean worker: {(wmax - wmean).mean():.0f} cycles per step")
which = wk.argmax(axis=1) + 1
print("  slowest worker by index (share of steps):",
      " ".join(f"{i}:{100.0 * (which == i).mean():.0f}%" for i in range(1, 16)))
