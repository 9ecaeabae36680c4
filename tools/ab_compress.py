#!/usr/bin/env python3
"""Interleaved A/B timing of the compress (or, with AB_MODE=decompress, the
decompress) kernel across library builds: one process, same device
(cdna_hip_programming.md §5.4 rule 24).
usage: [AB_MODE=decompress] ab_compress.py KIND N COUNT ROUNDS LIB_A LIB_B [...]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def load(path):
    L = ctypes.CDLL(path)
    vp, u32 = ctypes.c_void_p, ctypes.c_uint32
    L.lzf_gpu_compress_batch.argtypes = [vp, vp, vp, vp, vp, vp, vp, u32, u32, vp]
    L.lzf_gpu_decompress_batch.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, u32, u32, vp]
    L.lzf_gpu_synth_fill.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                     u32, u32, vp, vp]
    return L


def main():
    kind, n, count, rounds = (int(x, 0) for x in sys.argv[1:5])
    libs = [(p, load(p)) for p in sys.argv[5:]]
    dev = "cuda"
    src = torch.empty(count * n, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    h = ctypes.c_void_p(s.cuda_stream)
    seed = int(os.environ.get("AB_SEED", "0x5EED0002"), 0)
    libs[0][1].lzf_gpu_synth_fill(kind, seed, 0, 1, count, n, ctypes.c_void_p(src.data_ptr()), h)
    off = torch.arange(count, dtype=torch.int64, device=dev) * n
    ln = torch.full((count,), n, dtype=torch.int32, device=dev)
    cap = torch.full((count,), n - 4, dtype=torch.int32, device=dev)
    outs = []
    res = {p: [] for p, _ in libs}
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    if os.environ.get("AB_MODE") == "decompress":
        comp = torch.empty(count * n, dtype=torch.uint8, device=dev)
        cl = torch.zeros(count, dtype=torch.int32, device=dev)
        libs[0][1].lzf_gpu_compress_batch(P(src), P(off), P(ln), P(comp), P(off), P(cap), P(cl), count, n, h)
        dcap = torch.full((count,), n, dtype=torch.int32, device=dev)
        for r in range(rounds + 1):
            for p, L in libs:
                out = torch.zeros(count * n, dtype=torch.uint8, device=dev)
                ol = torch.zeros(count, dtype=torch.int32, device=dev)
                er = torch.zeros(count, dtype=torch.int32, device=dev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                rc = L.lzf_gpu_decompress_batch(P(comp), P(off), P(cl), P(out), P(off), P(dcap), P(ol),
                                                P(er), count, n, h)
                e1.record(s)
                torch.cuda.synchronize()
                assert rc == 0
                if r:
                    res[p].append(e0.elapsed_time(e1))
                if r == 1:
                    ok = cl > 0
                    good = bool(((ol == n) | ~ok).all()) and bool((er[ok] == 0).all())
                    for r0 in range(0, count, 1 << 16):      # every byte of every value
                        r1 = min(count, r0 + (1 << 16))
                        good = good and not bool(((out.view(count, n)[r0:r1] != src.view(count, n)[r0:r1])
                                                  .any(dim=1) & ok[r0:r1]).any())
                    print(f"{os.path.basename(p)} round trip ok: {good}", flush=True)
        for p, t in res.items():
            t.sort()
            print(f"{os.path.basename(p):28s} median {t[len(t) // 2]:8.2f} ms  min {t[0]:8.2f}  "
                  f"{count * n / t[len(t) // 2] / 1e6:7.2f} GB/s (decompress, output bytes)")
        return
    for r in range(rounds + 1):
        for p, L in libs:
            out = torch.empty(count * n, dtype=torch.uint8, device=dev)
            ol = torch.zeros(count, dtype=torch.int32, device=dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            rc = L.lzf_gpu_compress_batch(P(src), P(off), P(ln), P(out), P(off), P(cap), P(ol), count, n, h)
            e1.record(s)
            torch.cuda.synchronize()
            assert rc == 0
            if r:
                res[p].append(e0.elapsed_time(e1))
            if r == 1:
                outs.append((p, ol.clone(), out))
    base = outs[0]
    for p, ol, out in outs[1:]:
        same = torch.equal(ol, base[1])
        # every stream byte of every value (masked by its length), in slices
        for r0 in range(0, count, 1 << 14):
            if not same:
                break
            r1 = min(count, r0 + (1 << 14))
            mask = torch.arange(n, device=dev).unsqueeze(0) < ol[r0:r1].unsqueeze(1)
            same = not bool(((out.view(count, n)[r0:r1] != base[2].view(count, n)[r0:r1]) & mask).any())
        print(f"{os.path.basename(p)} output identical to {os.path.basename(base[0])}: {same}", flush=True)
    for p, t in res.items():
        t.sort()
        print(f"{os.path.basename(p):28s} median {t[len(t) // 2]:8.2f} ms  min {t[0]:8.2f}  "
              f"{count * n / t[len(t) // 2] / 1e6:7.2f} GB/s")


if __name__ == "__main__":
    main()
