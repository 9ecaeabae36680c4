"""Child process of tests/test_host_paths.py: the host-memory batch calls
under the device plan in LZF_GPU_DEVICES (read once per process), checked
bit-for-bit -- mixed values against the oracle, and the first 262 144 values
of BASELINE configs[1] against the reference's whole-batch digest
(tests/golden/digests.json) -- on the staged path and on registered arenas.
Prints one JSON line."""
import json
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime in the process)

import gibson_amd  # noqa: E402
from tests.digest import batch_digest  # noqa: E402
from tests.oracle_lib import Oracle, _SYN, synth  # noqa: E402


def aligned(nbytes):
    """zeroed bytes at a page boundary (a registered range owns its pages)"""
    raw = np.zeros(nbytes + 8192, np.uint8)
    k = (-raw.ctypes.data) % 4096
    return raw[k:k + nbytes]


def mixed_case(oracle, register):
    rnd = random.Random(23)
    count = 3000
    sizes = [rnd.choice([4096, 16384, rnd.randint(0, 20000)]) for _ in range(count)]
    order = list(range(count))
    rnd.shuffle(order)
    pos, offs = 0, [0] * count
    for i in order:
        offs[i] = pos
        pos += sizes[i] + rnd.randint(0, 40)
    arena = aligned(pos + 64)
    for i in range(count):
        arena[offs[i]:offs[i] + sizes[i]] = np.frombuffer(synth(i % 6, 0x5EED00C0, i, sizes[i]), np.uint8)
    off = np.array(offs, dtype=np.uint64)
    ln = np.array(sizes, dtype=np.uint32)
    cap = np.maximum(ln.astype(np.int64) - 4, 0).astype(np.uint32)
    out = aligned(pos + 64)
    olen = np.zeros(count, np.uint32)
    dec = aligned(pos + 64)
    regs = (arena, out, dec) if register else ()
    for a in regs:
        gibson_amd.host_register(a)
    try:
        gibson_amd.host_compress_batch(arena, off, ln, out, off, cap, olen)
        spread_c = gibson_amd.host_last_spread()
        bad = 0
        for i in range(count):
            v = bytes(arena[offs[i]:offs[i] + sizes[i]])
            exp = oracle.compress(v, int(cap[i])) if sizes[i] and cap[i] else None
            got = bytes(out[offs[i]:offs[i] + olen[i]]) if olen[i] else None
            bad += got != exp
        ok = olen > 0
        dl = np.zeros(int(ok.sum()), np.uint32)
        er = np.zeros(int(ok.sum()), np.int32)
        gibson_amd.host_decompress_batch(out, off[ok], olen[ok], dec, off[ok], ln[ok], dl, er)
        rt = bool((dl == ln[ok]).all() and (er == 0).all())
        for i in np.nonzero(ok)[0]:
            rt &= bytes(dec[offs[i]:offs[i] + sizes[i]]) == bytes(arena[offs[i]:offs[i] + sizes[i]])
    finally:
        for a in regs:
            gibson_amd.host_unregister(a)
    return {"values": count, "mismatches": int(bad), "roundtrip": bool(rt), "spread": spread_c}


def digest_case(register):
    kind, seed, n, count = 1, 0x5EED0002, 4096, 262144
    arena = aligned(count * n)
    _SYN.synth_fill(kind, seed, 0, count, n, arena.ctypes.data)
    off = np.arange(count, dtype=np.uint64) * n
    ln = np.full(count, n, np.uint32)
    cap = np.full(count, n - 4, np.uint32)
    out = aligned(count * n)
    olen = np.zeros(count, np.uint32)
    regs = (arena, out) if register else ()
    for a in regs:
        gibson_amd.host_register(a)
    try:
        gibson_amd.host_compress_batch(arena, off, ln, out, off, cap, olen)
        spread = gibson_amd.host_last_spread()
    finally:
        for a in regs:
            gibson_amd.host_unregister(a)
    return {"digest": batch_digest(out, n, olen), "spread": spread}


def main():
    oracle = Oracle()
    res = {"plan": gibson_amd.device_plan(), "split": gibson_amd.host_split_policy()}
    for reg in (False, True):
        tag = "registered" if reg else "staged"
        res["mixed_" + tag] = mixed_case(oracle, reg)
        res["config1_" + tag] = digest_case(reg)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
