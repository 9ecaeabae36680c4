#!/usr/bin/env python3
"""Compress time by batch size for the lane and window generations: where
does the lane generation start to pay?  usage: crossover.py [KIND N [MAX_COUNT]]
(default json4k: 1 4096).  The lane parse runs
one value per lane, so a small batch leaves the GPU mostly idle while each
lane walks its whole value."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gibson_amd  # noqa: E402

kind = int(sys.argv[1]) if len(sys.argv) > 1 else 1
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
N = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20
os.environ["LZF_GPU_LANE_MIN"] = "0"
dev = torch.device("cuda")
src = torch.empty(N * n, dtype=torch.uint8, device=dev)
gibson_amd.synth_fill(kind, 0x5EED0002, 0, 1, N, n, src)
off = torch.arange(N, dtype=torch.int64, device=dev) * n
ln = torch.full((N,), n, dtype=torch.int32, device=dev)
cap = torch.full((N,), n - 4, dtype=torch.int32, device=dev)
out = torch.empty(N * n, dtype=torch.uint8, device=dev)
olen = torch.zeros(N, dtype=torch.int32, device=dev)


def t(count, gen):
    if gen == "window":
        os.environ["LZF_GPU_KERNEL"] = "window"
    else:
        os.environ.pop("LZF_GPU_KERNEL", None)
    ts = []
    for _ in range(4):
        torch.cuda.synchronize()
        a = time.perf_counter()
        gibson_amd.compress_batch(src, off[:count], ln[:count], out, off[:count], cap[:count], olen[:count], n)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - a)
    return sorted(ts)[1] * 1e3


counts = [int(c) for c in os.environ["XO_COUNTS"].split(",")] if os.environ.get("XO_COUNTS") else \
    [1 << 10, 1 << 12, 1 << 14, 1 << 16, 1 << 17, 1 << 18, 1 << 19, 1 << 20]
for count in counts:
    if count > N:
        break
    print(f"{count:8d} values: lane {t(count, 'lane'):8.2f} ms   window {t(count, 'window'):8.2f} ms", flush=True)
