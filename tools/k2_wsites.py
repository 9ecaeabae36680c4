#!/usr/bin/env python3
"""How often a WAVE of the lane parse runs each section (diagnostic build
gibson_amd/liblzf_hip_ws.so, -DK2_WAVE_SITES), per wave: the lane parse is
issue-bound on mixed data (profiles/r06/n/mix_mixed16k.txt), and a section
costs its instructions once per wave pass whatever its active lanes.
usage: k2_wsites.py KIND SEED N COUNT"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["LZF_HIP_LIB"] = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gibson_amd",
                                         "liblzf_hip_ws.so")
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
L.lzf_gpu_debug_sites(buf, 1)
gibson_amd.compress_batch(src, off, ln, out, off, cap, olen, n)
torch.cuda.synchronize()
L.lzf_gpu_debug_sites(buf, 0)
waves = (count + 63) // 64
names = ["wave iterations", "STEP", "STEP block load", "RESOLVE test", "DECIDE", "DECIDE literal",
         "free-literal path", "fm mask", "free-literal trip", "DECIDE match", "EXTEND", "EMIT",
         "EMIT multiword", "-", "-", "-"]
print(f"kind {kind} n {n} count {count}: per wave ({waves} waves)")
for i, nm in enumerate(names):
    if nm != "-":
        print(f"  {nm:20s} {buf[i] / waves:10.1f}")
