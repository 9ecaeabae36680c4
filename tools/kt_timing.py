#!/usr/bin/env python3
"""Per-phase cycles of lzf_cand_table_kernel (diagnostic build
gibson_amd/liblzf_hip_timing.so, -DKT_TIMING), averaged per wave-step.
usage: kt_timing.py KIND N COUNT"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("LZF_HIP_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gibson_amd",
                                         "liblzf_hip_timing.so"))
os.environ.setdefault("LZF_GPU_TABLE_STAGE", "1")
os.environ.setdefault("LZF_GPU_LANE_MIN", "0")
import torch  # noqa: E402

import gibson_amd  # noqa: E402

kind, n, count = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
L = gibson_amd.lib()
L.lzf_gpu_debug_kt.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
src = torch.empty(count * n, dtype=torch.uint8, device="cuda")
gibson_amd.synth_fill(kind, 0x5EED0003, 0, 1, count, n, src)
off = torch.arange(count, dtype=torch.int64, device="cuda") * n
ln = torch.full((count,), n, dtype=torch.int32, device="cuda")
cap = torch.full((count,), n - 4, dtype=torch.int32, device="cuda")
out = torch.empty(count * n, dtype=torch.uint8, device="cuda")
olen = torch.zeros(count, dtype=torch.int32, device="cuda")
gibson_amd.compress_batch(src, off, ln, out, off, cap, olen, n)
torch.cuda.synchronize()
L.lzf_gpu_debug_kt(buf, 1)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
gibson_amd.compress_batch(src, off, ln, out, off, cap, olen, n)
e1.record()
torch.cuda.synchronize()
L.lzf_gpu_debug_kt(buf, 0)
v = list(buf)
nw = int(os.environ.get("KT_WIN", "15"))  # worker waves per workgroup
steps = v[7] / (nw + 1)  # steps counted by every wave
names = ["B (table wave)", "table wave barrier", "C2", "C1", "A", "worker loads", "worker barrier"]
print(f"kernel {e0.elapsed_time(e1):.2f} ms, {steps:.0f} workgroup-steps")
for i, nm in enumerate(names):
    per = v[i] / steps / (1 if i < 2 else nw)
    print(f"  {nm:22s} {per:9.1f} cycles per step (per wave)")
if v[8]:   # busy cycles before the barrier: the slowest worker and the mean worker, per step
    print(f"  workers' busy time per step: slowest {v[8] / steps:9.1f}, mean {v[9] / steps:9.1f} cycles")
