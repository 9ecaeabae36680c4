#!/usr/bin/env python3
"""Compress time of the table generation against the batch size: the whole
launch and the cand kernel alone (LZF_GPU_TABLE_STAGE=1), so the parse is the
difference.  Tells whether the one-lane-per-value parse is bound by one
value's serial latency (time flat in the count) or by the machine (time
proportional to it).  usage: parse_scaling.py KIND N COUNT [COUNT ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("LZF_GPU_LANE_MIN", "0")
import torch  # noqa: E402

import gibson_amd  # noqa: E402


def timed(fn, reps=3):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    kind, n = int(sys.argv[1]), int(sys.argv[2])
    counts = [int(x) for x in sys.argv[3:]]
    top = max(counts)
    src = torch.empty(top * n, dtype=torch.uint8, device="cuda")
    gibson_amd.synth_fill(kind, 0x5EED0003, 0, 1, top, n, src)
    out = torch.empty(top * n, dtype=torch.uint8, device="cuda")
    for c in counts:
        off = torch.arange(c, dtype=torch.int64, device="cuda") * n
        ln = torch.full((c,), n, dtype=torch.int32, device="cuda")
        cap = torch.full((c,), n - 4, dtype=torch.int32, device="cuda")
        olen = torch.zeros(c, dtype=torch.int32, device="cuda")
        run = lambda: gibson_amd.compress_batch(src, off, ln, out, off, cap, olen, n)  # noqa: E731
        run()
        torch.cuda.synchronize()
        full = timed(run)
        os.environ["LZF_GPU_TABLE_STAGE"] = "1"
        cand = timed(run)
        del os.environ["LZF_GPU_TABLE_STAGE"]
        print(f"count {c:7d}: compress {full:8.2f} ms  cand {cand:7.2f} ms  parse {full - cand:7.2f} ms  "
              f"({full / c * 1e3:.3f} us/value)  {gibson_amd.kernel_info()}", flush=True)


if __name__ == "__main__":
    main()
