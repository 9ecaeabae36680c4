#!/usr/bin/env python3
"""Generate the golden LZF fixtures from the compiled reference codec.

Run in the build container (needs /root/reference):
    make -C oracle ref && python tests/golden/make_golden.py

Inputs come from the synthetic generators (gibson_amd/csrc/synth.h, host
build libgibson_synth.so) or are literal byte strings; outputs come from
oracle/_ref/liblzf_ref.so, i.e. /root/reference/src/lzf_c.c + lzf_d.c compiled
by oracle/Makefile.  Only data is written: inputs (as generator coordinates
or hex), output lengths, errno values, sha256 digests and, for small cases,
full output hex.

Files:
  kat.json     known-answer vectors of SURVEY.md §8(c), checked against _ref
  corpus.json  randomized compress cases over kinds x sizes x out_len regimes
               (incl. the exact success/failure boundary), plus decoder cases
               (valid streams, truncations, corruptions, tight out_len)
  config0.json BASELINE configs[0]: the 64 KiB text value at seed 0x5EED0001,
               its reference stream (sha256, length) and round trip
  digests.json full-batch digests of the BASELINE configs' generators: the
               first 64 K values of configs[1..4] (and all 256 K of configs[2])
               compressed by the reference at out_len = n-4 (src/query.c:385);
               digest = sha256 over the values in order of (u32 LE length ||
               stream), a length of 0 = does not fit (tests/digest.py)
"""
import ctypes
import errno
import hashlib
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "liblzf_ref.so"), use_errno=True)
SYN = ctypes.CDLL(os.path.join(ROOT, "gibson_amd", "libgibson_synth.so"))
for f in (REF.ref_lzf_compress, REF.ref_lzf_decompress):
    f.restype = ctypes.c_uint
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p, ctypes.c_uint]
SYN.synth_fill.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                           ctypes.c_uint32, ctypes.c_void_p]


def synth(kind, seed, index, n):
    buf = ctypes.create_string_buffer(max(n, 1))
    SYN.synth_fill(kind, seed, index, 1, n, buf)
    return buf.raw[:n]


def ref_compress(data, out_len):
    src = ctypes.create_string_buffer(data + b"\0" * 8, len(data) + 8)
    dst = ctypes.create_string_buffer(out_len + 16)
    r = REF.ref_lzf_compress(src, len(data), dst, out_len)
    return dst.raw[:r] if r else None


def ref_decompress(data, out_len):
    # the reference reads one control byte even for in_len == 0
    src = ctypes.create_string_buffer(data + b"\xff", len(data) + 1)
    dst = ctypes.create_string_buffer(out_len + 16)
    ctypes.set_errno(0)
    r = REF.ref_lzf_decompress(src, len(data), dst, out_len)
    e = ctypes.get_errno() if r == 0 else 0
    return r, e, (dst.raw[:r] if r else b"")


def sha(b):
    return hashlib.sha256(b).hexdigest()[:16]


def kat():
    cases = []
    # SURVEY §8(c) known answers
    z39 = b"Z" + b"abcdefghijklmnopqrs" * 2
    for data, out_len in [(z39, 1000), (z39, 35), (b"x", 3), (b"x", 4), (b"x", 1), (b"", 16),
                          (b"ab", 5), (b"abc", 6), (b"aaaaaaaa", 12), (b"a" * 300, 296),
                          (b"abcabcabcabcabcabcabc", 100)]:
        r = ref_compress(data, out_len)
        cases.append({"op": "compress", "in_hex": data.hex(), "out_len": out_len,
                      "result": len(r) if r else 0, "out_hex": r.hex() if r else ""})
    for data, out_len in [(b"\x02abc", 2), (b"\x05abc", 100), (b"\x00a\x20\x05", 100),
                          (b"\x00a\x20\x05", 2), (b"\x00z\xa0\x00", 100), (b"\x00z\xa0\x00", 8),
                          (b"\x00z\xa0\x00", 7), (b"\x00z\xe0", 100), (b"\x00z\xe0\x01", 100),
                          (b"\x00z\xe0\x01\x00", 100), (b"\x20", 100), (b"\x1f" + b"q" * 32, 32),
                          (b"\x1f" + b"q" * 31, 100)]:
        r, e, out = ref_decompress(data, out_len)
        cases.append({"op": "decompress", "in_hex": data.hex(), "out_len": out_len,
                      "result": r, "errno": e, "out_hex": out.hex()})
    # the documented quirk: a 19-byte ref e0 0a 12 at the end of z39
    assert cases[0]["out_hex"].endswith("e00a12"), cases[0]
    return cases


KINDS = [0, 1, 2, 3, 4, 5]


def corpus():
    rnd = random.Random(0x60D)
    comp = []
    sizes = list(range(1, 41)) + [41, 63, 64, 65, 100, 255, 256, 257, 1000, 1024, 4095, 4096,
                                  4097, 8192, 16384, 65535, 65536, 65537, 100000, 262144]
    for kind in KINDS:
        for n in sizes:
            reps = 3 if n <= 4096 else 1
            for rep in range(reps):
                seed = 0x5EED0000 + kind * 97 + rep
                index = rnd.randrange(1 << 20)
                data = synth(kind, seed, index, n)
                big = n + n // 16 + 64
                full = ref_compress(data, big)
                F = len(full) if full else 0
                outs = {n - 4 if n > 4 else 1, big, rnd.randint(1, big)}
                if F:
                    outs |= {max(1, F + d) for d in (-1, 0, 1, 2, 3, 4)}
                for out_len in sorted(outs):
                    r = ref_compress(data, out_len)
                    rec = {"kind": kind, "seed": seed, "index": index, "n": n,
                           "in_sha": sha(data), "out_len": out_len,
                           "result": len(r) if r else 0, "out_sha": sha(r) if r else ""}
                    if n <= 48 and r:
                        rec["in_hex"] = data.hex()
                        rec["out_hex"] = r.hex()
                    comp.append(rec)
    dec = []
    for kind in KINDS:
        for n in (1, 2, 3, 7, 40, 300, 4096, 8192):
            seed = 0x5EED1000 + kind
            index = rnd.randrange(1 << 20)
            data = synth(kind, seed, index, n)
            stream = ref_compress(data, n + n // 16 + 64)
            base = {"kind": kind, "seed": seed, "index": index, "n": n,
                    "stream_len": len(stream), "stream_sha": sha(stream)}
            cases = [(stream, n, {}), (stream, n - 1, {}), (stream, n + 100, {})]
            cuts = range(len(stream)) if len(stream) <= 400 else sorted(rnd.sample(range(len(stream)), 24))
            for cut in cuts:
                cases.append((stream[:cut], n, {"cut": cut}))
            for k in range(6):
                bad = bytearray(stream)
                pos = rnd.randrange(len(bad))
                bad[pos] = rnd.randrange(256)
                cases.append((bytes(bad), n + 64, {"flip": [pos, bad[pos]]}))
            for s, out_len, mod in cases:
                out_len = max(out_len, 0)
                r, e, out = ref_decompress(s, out_len)
                rec = dict(base)
                rec.update(mod)
                rec.update({"out_len": out_len, "result": r, "errno": e,
                            "out_sha": sha(out) if r else ""})
                dec.append(rec)
    for k in range(300):
        s = bytes(rnd.randrange(256) for _ in range(rnd.randint(1, 40)))
        out_len = rnd.choice([0, 1, 5, 40, 300, 10000])
        r, e, out = ref_decompress(s, out_len)
        dec.append({"kind": -1, "tag": "random", "in_hex": s.hex(), "out_len": out_len,
                    "result": r, "errno": e, "out_sha": sha(out) if r else ""})
    return comp, dec


# (BASELINE config, kind, seed, n, count) -- tests/digest.py holds the same
DIGEST_CONFIGS = [
    (1, 1, 0x5EED0002, 4096, 65536),
    (2, 2, 0x5EED0003, 65536, 65536),
    (2, 2, 0x5EED0003, 65536, 262144),
    (3, 0, 0x5EED0004, 8192, 65536),
    (4, 3, 0x5EED0005, 16384, 65536),
    # the production routes at their real batch sizes (above
    # gibson_amd/csrc/lzf_api.cpp lane_min_count, the routing's batch
    # thresholds): both take the lane generation, the stream cand kernel
    # (lzf_stream.hip) and the lane parse
    (1, 1, 0x5EED0002, 4096, 262144),
    (4, 3, 0x5EED0005, 16384, 131072),
    # round 5: the configs' real counts -- all of configs[1], the first
    # 1 M-value chunk of configs[4] (the chunk bench.py runs), and 1 M values
    # of configs[3] with the reference decoder's output digest (ROUNDTRIP)
    (1, 1, 0x5EED0002, 4096, 1048576),
    (4, 3, 0x5EED0005, 16384, 1048576),
    (3, 0, 0x5EED0004, 8192, 1048576),
]
# configs whose record also holds decoded_sha256: sha256 over the values in
# order of (u32 LE decoded length || the reference decoder's output), the
# length 0 for a value that did not compress
ROUNDTRIP = {(0, 0x5EED0004, 8192, 1048576)}
# round 6: the rest of the configs' real counts, in 1 M-value chunks starting
# at `first` -- configs[3]'s other 7 M values (with the decoder's output
# digest) and configs[4]'s other three 1 M chunks
# (BASELINE config, kind, seed, n, first, count)
DIGEST_CHUNKS = ([(3, 0, 0x5EED0004, 8192, k << 20, 1 << 20) for k in range(1, 8)] +
                 [(4, 3, 0x5EED0005, 16384, k << 20, 1 << 20) for k in range(1, 4)])
ROUNDTRIP_KINDS = {(0, 0x5EED0004, 8192)}


def digests(have=()):
    """reference digests of DIGEST_CONFIGS, skipping the (kind, seed, n,
    count) keys in ``have``"""
    import numpy as np
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libref_batch.so"))
    lib.ref_batch_compress.restype = ctypes.c_int
    lib.ref_batch_compress.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                       ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_int]
    lib.ref_batch_roundtrip.restype = ctypes.c_int
    lib.ref_batch_roundtrip.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                        ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    res = []
    todo = [(cfg, kind, seed, n, 0, count) for cfg, kind, seed, n, count in DIGEST_CONFIGS
            if (kind, seed, n, count) not in have]
    todo += [(cfg, kind, seed, n, f0, count) for cfg, kind, seed, n, f0, count in DIGEST_CHUNKS
             if (kind, seed, n, f0, count) not in have]
    for cfg, kind, seed, n, f0, count in todo:
        rt = (kind, seed, n, count) in ROUNDTRIP or (f0 and (kind, seed, n) in ROUNDTRIP_KINDS)
        h, hd = hashlib.sha256(), hashlib.sha256()
        chunk = max(1, min(count, (512 << 20) // n))
        out = np.empty(chunk * n, np.uint8)
        lens = np.empty(chunk, np.uint32)
        dec = np.empty(chunk * n, np.uint8) if rt else None
        dlens = np.empty(chunk, np.uint32) if rt else None
        total = comp = 0
        for first in range(0, count, chunk):
            m = min(chunk, count - first)
            if rt:
                rc = lib.ref_batch_roundtrip(kind, seed, f0 + first, m, n, 4, out.ctypes.data, lens.ctypes.data,
                                             dec.ctypes.data, dlens.ctypes.data, os.cpu_count() or 1)
            else:
                rc = lib.ref_batch_compress(kind, seed, f0 + first, m, n, 4, out.ctypes.data, lens.ctypes.data,
                                            os.cpu_count() or 1)
            assert rc == 0
            for k in range(m):
                ln = int(lens[k])
                h.update(ln.to_bytes(4, "little"))
                h.update(out[k * n:k * n + ln].data)
                comp += ln
                if rt:
                    dl = int(dlens[k])
                    hd.update(dl.to_bytes(4, "little"))
                    hd.update(dec[k * n:k * n + dl].data)
            total += m
        rec = {"config": cfg, "kind": kind, "seed": seed, "n": n, "first": f0, "count": count,
               "out_len": "n-4", "sha256": h.hexdigest(), "comp_bytes": comp}
        if rt:
            rec["decoded_sha256"] = hd.hexdigest()
            rec["decode_out_len"] = "n"
        res.append(rec)
        print("digest", cfg, n, f0, count, h.hexdigest()[:16], comp / (count * n), flush=True)
    return res


def config0():
    """BASELINE configs[0]: one 64 KiB Zipf-text value (SYN_TEXT, seed
    0x5EED0001, index 0) through the reference lzf_compress at out_len = n-4
    (src/query.c:385) and back through lzf_decompress at the server's
    out_len = maxrequestsize (4 MiB, src/default.h:45; src/net.c:1234)."""
    n = 65536
    data = synth(0, 0x5EED0001, 0, n)
    stream = ref_compress(data, n - 4)
    assert stream
    r, e, out = ref_decompress(stream, 4 << 20)
    assert r == n and e == 0 and out == data          # the reference's own round trip
    return {"config": 0, "kind": 0, "seed": 0x5EED0001, "index": 0, "n": n,
            "in_sha256": hashlib.sha256(data).hexdigest(), "out_len": n - 4,
            "stream_len": len(stream), "stream_sha256": hashlib.sha256(stream).hexdigest(),
            "decode_out_len": 4 << 20, "decode_result": r, "decode_errno": e}


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    if len(sys.argv) > 1 and sys.argv[1] == "config0":
        c0 = config0()
        with open(os.path.join(here, "config0.json"), "w") as f:
            json.dump({"generator": "tests/golden/make_golden.py config0",
                       "source": "oracle/_ref/liblzf_ref.so (reference lzf_c.c, lzf_d.c)", **c0}, f, indent=1)
        print("config0", c0["stream_len"], c0["stream_sha256"][:16])
        return 0
    if len(sys.argv) > 1 and sys.argv[1] == "digests-add":
        # append the DIGEST_CONFIGS records digests.json does not hold yet
        path = os.path.join(here, "digests.json")
        with open(path) as f:
            doc = json.load(f)
        have = {(d["kind"], d["seed"], d["n"], d["count"]) for d in doc["digests"] if not d.get("first")}
        have |= {(d["kind"], d["seed"], d["n"], d["first"], d["count"]) for d in doc["digests"] if d.get("first")}
        doc["digests"] += digests(have)
        with open(path, "w") as f:
            json.dump(doc, f, indent=1)
        return 0
    if len(sys.argv) > 1 and sys.argv[1] == "digests":
        with open(os.path.join(here, "digests.json"), "w") as f:
            json.dump({"generator": "tests/golden/make_golden.py digests",
                       "source": "oracle/_ref/libref_batch.so (reference lzf_c.c)",
                       "record": "sha256 over values in order of u32 LE length || stream",
                       "digests": digests()}, f, indent=1)
        return 0
    k = kat()
    with open(os.path.join(here, "kat.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "source": "oracle/_ref/liblzf_ref.so",
                   "cases": k}, f, indent=0)
    c, d = corpus()
    with open(os.path.join(here, "digests.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py digests",
                   "source": "oracle/_ref/libref_batch.so (reference lzf_c.c)",
                   "record": "sha256 over values in order of u32 LE length || stream",
                   "digests": digests()}, f, indent=1)
    with open(os.path.join(here, "corpus.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "source": "oracle/_ref/liblzf_ref.so",
                   "E2BIG": errno.E2BIG, "EINVAL": errno.EINVAL,
                   "compress": c, "decompress": d}, f, separators=(",", ":"))
    print("kat", len(k), "compress", len(c), "decompress", len(d))


if __name__ == "__main__":
    sys.exit(main())
