#!/usr/bin/env python3
"""Pipe decoder phase balance (diagnostic CD_TIMING builds): decode a batch of
KIND/N values with each library and print producer / consumer busy and
barrier-wait cycles per round.   usage: dec_tstat.py KIND N COUNT LIB..."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    kind, n, count = (int(x, 0) for x in sys.argv[1:4])
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    vp, u32 = ctypes.c_void_p, ctypes.c_uint32
    dev = "cuda"
    src = torch.empty(count * n, dtype=torch.uint8, device=dev)
    off = torch.arange(count, dtype=torch.int64, device=dev) * n
    ln = torch.full((count,), n, dtype=torch.int32, device=dev)
    cap = torch.full((count,), n - 4, dtype=torch.int32, device=dev)
    comp = torch.empty(count * n, dtype=torch.uint8, device=dev)
    cl = torch.zeros(count, dtype=torch.int32, device=dev)
    h = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    first = True
    for path in sys.argv[4:]:
        L = ctypes.CDLL(path)
        L.lzf_gpu_compress_batch.argtypes = [vp, vp, vp, vp, vp, vp, vp, u32, u32, vp]
        L.lzf_gpu_decompress_batch.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, u32, u32, vp]
        L.lzf_gpu_synth_fill.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                         u32, u32, vp, vp]
        if first:
            L.lzf_gpu_synth_fill(kind, 0x5EED0002, 0, 1, count, n, P(src), h)
            L.lzf_gpu_compress_batch(P(src), P(off), P(ln), P(comp), P(off), P(cap), P(cl), count, n, h)
            first = False
        out = torch.zeros(count * n, dtype=torch.uint8, device=dev)
        ol = torch.zeros(count, dtype=torch.int32, device=dev)
        er = torch.zeros(count, dtype=torch.int32, device=dev)
        dcap = torch.full((count,), n, dtype=torch.int32, device=dev)
        st = (ctypes.c_ulonglong * 8)()
        timing = hasattr(L, "lzf_gpu_dec_tstat")
        for rep in range(2):    # the second run is the one reported
            if timing:
                L.lzf_gpu_dec_tstat(st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            L.lzf_gpu_decompress_batch(P(comp), P(off), P(cl), P(out), P(off), P(dcap), P(ol), P(er), count, n, h)
            e1.record()
            torch.cuda.synchronize()
            if timing:
                L.lzf_gpu_dec_tstat(st)
        print(os.path.basename(path), f"decode {e0.elapsed_time(e1):.2f} ms, {int((cl > 0).sum())} of {count} values compressed")
        if not timing:
            continue
        comp_bytes = int(cl.sum())
        rounds = comp_bytes / 128.0  # approx rounds (tokens starting in 128 input bytes)
        names = ["prod busy", "prod wait", "cons busy", "cons wait"]
        print(os.path.basename(path), " ".join(f"{nm} {st[i] / rounds:8.0f}" for i, nm in enumerate(names)),
              "cycles per ~round")
        if st[4] or st[5]:   # the producer's busy time split: discovery, decode
            print(f"  of the producer's busy time: discovery {st[4] / rounds:8.0f}, decode {st[5] / rounds:8.0f}, staging {st[6] / rounds:8.0f}")


if __name__ == "__main__":
    main()
