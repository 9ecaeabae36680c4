#!/usr/bin/env python3
"""Compress a synthetic batch (untimed) and decode it twice, for rocprofv3
counter runs of the decoder alone.  usage: decode_once.py KIND N COUNT"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gibson_amd  # noqa: E402

kind, n, count = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
dev = "cuda"
src = torch.empty(count * n, dtype=torch.uint8, device=dev)
gibson_amd.synth_fill(kind, 0x5EED0003, 0, 1, count, n, src)
off = torch.arange(count, dtype=torch.int64, device=dev) * n
ln = torch.full((count,), n, dtype=torch.int32, device=dev)
cap = torch.full((count,), n - 4, dtype=torch.int32, device=dev)
comp = torch.empty(count * n, dtype=torch.uint8, device=dev)
clen = torch.zeros(count, dtype=torch.int32, device=dev)
gibson_amd.compress_batch(src, off, ln, comp, off, cap, clen, n)
del src
dec = torch.empty(count * n, dtype=torch.uint8, device=dev)
dlen = torch.zeros(count, dtype=torch.int32, device=dev)
err = torch.zeros(count, dtype=torch.int32, device=dev)
for _ in range(2):
    gibson_amd.decompress_batch(comp, off, clen, dec, off, ln, dlen, err, n)
torch.cuda.synchronize()
print("decoded", int((dlen == n).sum()), "of", count)
