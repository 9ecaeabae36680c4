#!/usr/bin/env python3
"""Interleaved A/B of the compress kernels under different LZF_GPU_*
environment settings (the library reads them per launch), one process, one
device; outputs compared for identity against the first setting.
usage: ab_env.py KIND N COUNT ROUNDS 'VAR=x,VAR2=y' 'VAR=z' ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("LZF_GPU_LANE_MIN", "0")
import torch  # noqa: E402

import gibson_amd  # noqa: E402


def apply(setting, keys):
    for k in keys:
        os.environ.pop(k, None)
    for kv in filter(None, setting.split(",")):
        k, v = kv.split("=", 1)
        os.environ[k] = v


def main():
    kind, n, count, rounds = (int(x, 0) for x in sys.argv[1:5])
    settings = sys.argv[5:]
    keys = {kv.split("=", 1)[0] for s in settings for kv in filter(None, s.split(","))}
    src = torch.empty(count * n, dtype=torch.uint8, device="cuda")
    gibson_amd.synth_fill(kind, 0x5EED0003, 0, 1, count, n, src)
    off = torch.arange(count, dtype=torch.int64, device="cuda") * n
    ln = torch.full((count,), n, dtype=torch.int32, device="cuda")
    cap = torch.full((count,), n - 4, dtype=torch.int32, device="cuda")
    res = {s: [] for s in settings}
    outs = {}
    for r in range(rounds + 1):
        for st in settings:
            apply(st, keys)
            out = torch.zeros(count * n, dtype=torch.uint8, device="cuda")
            ol = torch.zeros(count, dtype=torch.int32, device="cuda")
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            gibson_amd.compress_batch(src, off, ln, out, off, cap, ol, n)
            e1.record()
            torch.cuda.synchronize()
            if r:
                res[st].append(e0.elapsed_time(e1))
            else:
                outs[st] = (ol, out, gibson_amd.kernel_info())
    base = settings[0]
    for st in settings[1:]:
        ol, out, _ = outs[st]
        b_ol, b_out, _ = outs[base]
        same = torch.equal(ol, b_ol)
        if same:
            o = out.view(count, n)
            bo = b_out.view(count, n)
            mask = torch.arange(n, device="cuda").unsqueeze(0) < ol.unsqueeze(1)
            same = bool(((o != bo) & mask).sum() == 0)
        print(f"[{st}] output identical to [{base}]: {same}", flush=True)
    for st, t in res.items():
        t.sort()
        print(f"[{st:40s}] median {t[len(t) // 2]:8.2f} ms  min {t[0]:8.2f}  ratio "
              f"{outs[st][0].sum().item() / (count * n):.4f}  {outs[st][2].split(' decompress')[0]}", flush=True)


if __name__ == "__main__":
    main()
