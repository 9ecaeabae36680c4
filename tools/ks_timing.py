#!/usr/bin/env python3
"""Per-phase cycles of lzf_cand_stream_kernel (diagnostic build
gibson_amd/liblzf_hip_kst.so, -DKS_TIMING), averaged per wave-step, for the
lane generation (LZF_GPU_LANE_STAGE=1) or, REC=1, the table generation's
record form (LZF_GPU_TCAND=stream, LZF_GPU_TABLE_STAGE=1).
usage: [REC=1] ks_timing.py KIND N COUNT"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["LZF_HIP_LIB"] = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gibson_amd",
                                         "liblzf_hip_kst.so")
os.environ.setdefault("LZF_GPU_LANE_MIN", "0")
if os.environ.get("REC") == "1":
    os.environ["LZF_GPU_KERNEL"] = "table"
    os.environ["LZF_GPU_TCAND"] = "stream"
    os.environ["LZF_GPU_TABLE_STAGE"] = "1"
else:
    os.environ["LZF_GPU_KERNEL"] = "lane"
    os.environ["LZF_GPU_LANE_STAGE"] = "1"
import torch  # noqa: E402

import gibson_amd  # noqa: E402

kind, n, count = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
L = gibson_amd.lib()
L.lzf_gpu_debug_ks.argtypes = [ctypes.c_void_p, ctypes.c_int]
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
L.lzf_gpu_debug_ks(buf, 1)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
gibson_amd.compress_batch(src, off, ln, out, off, cap, olen, n)
e1.record()
torch.cuda.synchronize()
L.lzf_gpu_debug_ks(buf, 0)
v = list(buf)
steps = v[8] / 16
names = ["table wave B", "table wave loads", "table wave barrier", "C2", "C1 (+Q)", "A", "worker loads+cursor",
         "worker barrier"]
print(f"kernel 1 {e0.elapsed_time(e1):.2f} ms, {steps:.0f} workgroup-steps, {gibson_amd.kernel_info()[:60]}")
for i, nm in enumerate(names):
    per = v[i] / steps / (1 if i < 3 else 15)
    print(f"  {nm:22s} {per:9.1f} cycles per step (per wave)")
