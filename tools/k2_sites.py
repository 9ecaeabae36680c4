#!/usr/bin/env python3
"""Per-site access counts of the lane parse kernel (diagnostic build
gibson_amd/liblzf_hip_sites.so, -DK2_COUNT_SITES), per value."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["LZF_HIP_LIB"] = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gibson_amd",
                                         "liblzf_hip_sites.so")
os.environ["LZF_GPU_LANE_PIPE"] = "0"
os.environ.setdefault("LZF_GPU_LANE_MIN", "0")   # the lane route at any batch size
import torch  # noqa: E402

import gibson_amd  # noqa: E402

kind, seed, n, count = int(sys.argv[1]), int(sys.argv[2], 0), int(sys.argv[3]), int(sys.argv[4])
L = gibson_amd.lib()
L.lzf_gpu_debug_sites.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
src = torch.empty(count * n, dtype=torch.uint8, device="cuda")
gibson_amd.synth_fill(kind, seed, 0, 1, count, n, src)
off = torch.arange(count, dtype=torch.int64, device="cuda") * n
ln = torch.full((count,), n, dtype=torch.int32, device="cuda")
cap = torch.full((count,), n - 4, dtype=torch.int32, device="cuda")
out = torch.empty(count * n, dtype=torch.uint8, device="cuda")
olen = torch.zeros(count, dtype=torch.int32, device="cuda")
gibson_amd.compress_batch(src, off, ln, out, off, cap, olen, n)
torch.cuda.synchronize()
L.lzf_gpu_debug_sites(buf, 1)
gibson_amd.compress_batch(src, off, ln, out, off, cap, olen, n)
torch.cuda.synchronize()
L.lzf_gpu_debug_sites(buf, 0)
names = ["lane-iterations", "C load", "C2 use", "bits load", "walk cand load", "eq3", "input window",
         "extend piece", "out dword", "free literal | wave: walk stops", "steps", "wave: windows", "wave: walk hops",
         "wave: long measures", "wave: truncations", "wave: orbit stops"]
for i, nm in enumerate(names):
    if nm != "-":
        print(f"{nm:16s} {buf[i] / count:10.1f} per value")
