#!/usr/bin/env python3
"""One warm-up and one timed compress of a synthetic batch (for rocprofv3
runs; the library is LZF_HIP_LIB if set).  usage: compress_once.py KIND N COUNT"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("LZF_GPU_LANE_MIN", "0")
import torch  # noqa: E402

import gibson_amd  # noqa: E402

kind, n, count = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
src = torch.empty(count * n, dtype=torch.uint8, device="cuda")
gibson_amd.synth_fill(kind, 0x5EED0003, 0, 1, count, n, src)
off = torch.arange(count, dtype=torch.int64, device="cuda") * n
ln = torch.full((count,), n, dtype=torch.int32, device="cuda")
cap = torch.full((count,), n - 4, dtype=torch.int32, device="cuda")
out = torch.empty(count * n, dtype=torch.uint8, device="cuda")
olen = torch.zeros(count, dtype=torch.int32, device="cuda")
for _ in range(2):
    gibson_amd.compress_batch(src, off, ln, out, off, cap, olen, n)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
gibson_amd.compress_batch(src, off, ln, out, off, cap, olen, n)
e1.record()
torch.cuda.synchronize()
print(f"compress {e0.elapsed_time(e1):.2f} ms  ratio {olen.sum().item() / (n * count):.4f}")
