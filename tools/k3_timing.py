#!/usr/bin/env python3
"""Counters of lzf_parse_rec_kernel (diagnostic build liblzf_hip_timing.so,
-DKT_TIMING): per value and per wave iteration.
usage: k3_timing.py KIND N COUNT"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("LZF_HIP_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                  "gibson_amd", "liblzf_hip_timing.so"))
os.environ.setdefault("LZF_GPU_LANE_MIN", "0")
import torch  # noqa: E402

import gibson_amd  # noqa: E402

kind, n, count = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
L = gibson_amd.lib()
L.lzf_gpu_debug_kt.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
src = torch.empty(count * n, dtype=torch.uint8, device="cuda")
gibson_amd.synth_fill(kind, int(os.environ.get("AB_SEED", "0x5EED0003"), 0), 0, 1, count, n, src)
off = torch.arange(count, dtype=torch.int64, device="cuda") * n
ln = torch.full((count,), n, dtype=torch.int32, device="cuda")
cap = torch.full((count,), n - 4, dtype=torch.int32, device="cuda")
out = torch.empty(count * n, dtype=torch.uint8, device="cuda")
olen = torch.zeros(count, dtype=torch.int32, device="cuda")
gibson_amd.compress_batch(src, off, ln, out, off, cap, olen, n)
torch.cuda.synchronize()
L.lzf_gpu_debug_kt(buf, 1)
gibson_amd.compress_batch(src, off, ln, out, off, cap, olen, n)
torch.cuda.synchronize()
L.lzf_gpu_debug_kt(buf, 0)
v = list(buf)[8:]
waves = (count + 63) // 64
print(f"per wave: {v[0] / waves:.0f} iterations, {v[1] / max(v[0], 1):.0f} cycles per iteration")
for i, nm in enumerate(["steps", "resolve tests", "bitmap words from scratch", "record hops", "extend pieces",
                        "block loads"], start=2):
    print(f"  {nm:26s} {v[i] / count:9.0f} per value")
