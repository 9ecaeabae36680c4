#!/usr/bin/env python3
"""Cycles per phase of the wave-form parse kernel (diagnostic build with
-DKW_PHASES, tools/build_variant.sh), per value."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
lib = sys.argv[5] if len(sys.argv) > 5 else "liblzf_hip_phases.so"
os.environ["LZF_HIP_LIB"] = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gibson_amd", lib)
os.environ["LZF_GPU_LANE_PIPE"] = "0"
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
names = ["stage", "decide", "orbit", "validate", "emit scan", "store+update", "orbit: walks", "orbit: long"]
tot = sum(buf[i] for i in range(8))
for i, nm in enumerate(names):
    print(f"{nm:18s} {buf[i] / count:12.0f} cycles/value  {100.0 * buf[i] / max(tot, 1):5.1f}%")
print(f"{'total':18s} {tot / count:12.0f}")
