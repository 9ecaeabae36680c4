#!/usr/bin/env python3
"""Does the decoder overlap with the compressor on two streams?  json4k
halves: compress(A) and decompress(B) back to back on one stream, then
concurrently on two (timing experiment for DESIGN.md §5)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gibson_amd  # noqa: E402

n, count = 4096, 1 << 19
dev = torch.device("cuda")
src = torch.empty(2 * count * n, dtype=torch.uint8, device=dev)
gibson_amd.synth_fill(1, 0x5EED0002, 0, 1, 2 * count, n, src)
off = torch.arange(count, dtype=torch.int64, device=dev) * n
ln = torch.full((count,), n, dtype=torch.int32, device=dev)
cap = torch.full((count,), n - 4, dtype=torch.int32, device=dev)
A, B = src[: count * n], src[count * n:]
cA = torch.empty(count * n, dtype=torch.uint8, device=dev)
cB = torch.empty(count * n, dtype=torch.uint8, device=dev)
lA = torch.zeros(count, dtype=torch.int32, device=dev)
lB = torch.zeros(count, dtype=torch.int32, device=dev)
dB = torch.empty(count * n, dtype=torch.uint8, device=dev)
dl = torch.zeros(count, dtype=torch.int32, device=dev)
de = torch.zeros(count, dtype=torch.int32, device=dev)
dcap = torch.full((count,), n, dtype=torch.int32, device=dev)
gibson_amd.compress_batch(B, off, ln, cB, off, cap, lB, n)
torch.cuda.synchronize()
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def run(concurrent):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        gibson_amd.compress_batch(A, off, ln, cA, off, cap, lA, n, s1)
        gibson_amd.decompress_batch(cB, off, lB, dB, off, dcap, dl, de, n, s2 if concurrent else s1)
        torch.cuda.synchronize()
    return (time.perf_counter() - t) / 3 * 1e3


for mode in (False, True, False, True):
    print(("two streams" if mode else "one stream "), f"{run(mode):.2f} ms")
