"""The CPU oracle against the reference's golden vectors (CPU only).

Pins oracle/lzf_oracle.c to the reference codec before it is trusted as the
checker of the HIP path: known answers, the randomized
corpus generated from the compiled reference (tests/golden/make_golden.py),
and -- where oracle/_ref was built in this container -- a live differential
run against the reference itself.
"""
import random

import pytest

from tests import oracle_lib
from tests.oracle_lib import sha16, synth


def test_kat(kat, oracle):
    for c in kat:
        data = bytes.fromhex(c["in_hex"])
        if c["op"] == "compress":
            r = oracle.compress(data, c["out_len"])
            assert (len(r) if r else 0) == c["result"], c
            if r:
                assert r.hex() == c["out_hex"], c
        else:
            out, e = oracle.decompress(data, c["out_len"])
            assert (len(out) if out else 0) == c["result"], c
            assert e == c["errno"], c
            if out:
                assert out.hex() == c["out_hex"], c


def test_quirk_19_byte_ref(oracle):
    # "Z"+X19+X19 emits a 19-byte ref e0 0a 12
    data = b"Z" + b"abcdefghijklmnopqrs" * 2
    assert oracle.compress(data, 1000).endswith(bytes.fromhex("e00a12"))


def test_corpus_compress(golden, oracle):
    cache = {}
    for c in golden["compress"]:
        key = (c["kind"], c["seed"], c["index"], c["n"])
        if key not in cache:
            cache[key] = synth(*key)
        data = cache[key]
        assert sha16(data) == c["in_sha"], "synthetic generator drifted"
        r = oracle.compress(data, c["out_len"])
        assert (len(r) if r else 0) == c["result"], c
        if r:
            assert sha16(r) == c["out_sha"], c
            if "out_hex" in c:
                assert r.hex() == c["out_hex"]


def _stream_for(c, oracle):
    data = synth(c["kind"], c["seed"], c["index"], c["n"])
    n = c["n"]
    stream = oracle.compress(data, n + n // 16 + 64)
    assert len(stream) == c["stream_len"] and sha16(stream) == c["stream_sha"]
    if "cut" in c:
        stream = stream[:c["cut"]]
    if "flip" in c:
        b = bytearray(stream)
        b[c["flip"][0]] = c["flip"][1]
        stream = bytes(b)
    return stream


def decoder_cases(golden, oracle):
    for c in golden["decompress"]:
        s = bytes.fromhex(c["in_hex"]) if "in_hex" in c else _stream_for(c, oracle)
        yield c, s


def test_corpus_decompress(golden, oracle):
    for c, s in decoder_cases(golden, oracle):
        out, e = oracle.decompress(s, c["out_len"])
        assert (len(out) if out else 0) == c["result"], c
        assert e == c["errno"], c
        if out:
            assert sha16(out) == c["out_sha"], c


@pytest.mark.skipif(oracle_lib.reference() is None, reason="oracle/_ref not built here")
def test_differential_vs_reference(oracle):
    ref = oracle_lib.reference()
    rnd = random.Random(1234)
    for it in range(3000):
        kind = rnd.randrange(6)
        n = rnd.choice([rnd.randint(1, 64), rnd.randint(1, 600), rnd.randint(1, 5000)])
        data = synth(kind, rnd.getrandbits(32), it, n)
        for out_len in (max(1, n - 4), n + 40, rnd.randint(1, n + 40)):
            assert oracle.compress(data, out_len) == ref.compress(data, out_len)
        s = ref.compress(data, n + n // 16 + 64)
        for out_len in (n, n - 1, rnd.randint(0, n + 5)):
            assert oracle.decompress(s, out_len) == ref.decompress(s, out_len)
        if len(s) > 2:
            b = bytearray(s)
            b[rnd.randrange(len(b))] = rnd.randrange(256)
            b = bytes(b[:rnd.randint(0, len(b))])
            assert oracle.decompress(b, n + 10) == ref.decompress(b, n + 10)


def test_oracle_matches_full_batch_digest():
    # the clean-room restatement against the reference's whole-batch digest of
    # BASELINE configs[1] (64 K JSON-like values of 4 KiB, out_len = n-4)
    import ctypes
    import json
    import os

    import numpy as np

    from tests.digest import batch_digest
    d = [x for x in json.load(open(os.path.join(oracle_lib.ROOT, "tests", "golden", "digests.json")))["digests"]
         if x["config"] == 1][0]
    n, count = d["n"], d["count"]
    syn = ctypes.CDLL(os.path.join(oracle_lib.ROOT, "gibson_amd", "libgibson_synth.so"))
    syn.synth_fill.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                               ctypes.c_uint32, ctypes.c_void_p]
    src = np.empty(count * n, np.uint8)
    syn.synth_fill(d["kind"], d["seed"], 0, count, n, src.ctypes.data)
    L = ctypes.CDLL(oracle_lib.ORACLE_SO)
    vp = ctypes.c_void_p
    L.oracle_compress_batch.argtypes = [vp, vp, vp, ctypes.c_uint32, vp, vp, vp, vp, ctypes.c_int]
    offs = np.arange(count, dtype=np.uint64) * n
    ln = np.full(count, n, np.uint32)
    cap = np.full(count, n - 4, np.uint32)
    out = np.empty(count * n, np.uint8)
    olen = np.empty(count, np.uint32)
    L.oracle_compress_batch(src.ctypes.data, offs.ctypes.data, ln.ctypes.data, count, out.ctypes.data,
                            offs.ctypes.data, cap.ctypes.data, olen.ctypes.data, 1)
    assert batch_digest(out, n, olen) == d["sha256"]


def test_oracle_config0_fixture(oracle):
    # BASELINE configs[0] (tests/golden/config0.json, from the reference):
    # the oracle's stream and round trip for the 64 KiB text value at seed
    # 0x5EED0001, out_len n-4 (src/query.c:385), decode at 4 MiB
    import hashlib
    import json
    import os
    with open(os.path.join(oracle_lib.ROOT, "tests", "golden", "config0.json")) as f:
        c = json.load(f)
    v = synth(c["kind"], c["seed"], c["index"], c["n"])
    assert hashlib.sha256(v).hexdigest() == c["in_sha256"]
    s = oracle.compress(v, c["out_len"])
    assert len(s) == c["stream_len"] and hashlib.sha256(s).hexdigest() == c["stream_sha256"]
    out, e = oracle.decompress(s, c["decode_out_len"])
    assert out == v and e == c["decode_errno"]


def test_far_route_predicate_and_flush_invariant():
    # the FAR decoder route (gibson_amd/csrc/lzf_decompress.hip, CD_FAR2)
    # decides "read this byte from HBM" with one add and one unsigned compare
    # on the owner token's info tInf (a back-reference's distance, 1..8192,
    # src/lzf_d.c:95; a literal's info has bit 31 set): restated here on every
    # distance and lane against the window rule it replaces (the source lies
    # more than the 4 KiB window behind the group's first byte), and the far
    # source checked to lie in output the 1 KiB flush units already stored
    import numpy as np
    window, unit = 4096, 1024
    omask = window - 1
    lane = np.arange(64, dtype=np.uint64)[None, :]
    t_ref = np.arange(1, 8193, dtype=np.uint64)[:, None]
    t_lit = (np.uint64(1 << 31) + np.arange(0, 4096, 7, dtype=np.uint64))[:, None]
    for gb in (64 * 64, 64 * 65, 64 * 128, 64 * 200, 64 * 1023):
        for tinf, lit in ((t_ref, False), (t_lit, True)):
            m = np.uint64(0xFFFFFFFF)
            o = np.uint64(gb) + lane
            so = (o - tinf) & m
            old = (not lit) & (so < gb) & (((np.uint64(gb) - so) & m) > window)
            new = np.broadcast_to(((tinf - lane - np.uint64(omask + 2)) & m) < np.uint64(8191 - omask), old.shape)
            # a reference before the output start fails in the round's decode
            # (EINVAL, src/lzf_d.c:127-130) and never reaches the output step
            valid = np.broadcast_to(lit | (tinf <= o), old.shape)
            assert np.array_equal(old[valid], new[valid]), gb
            if not lit:
                flushed = (gb // unit) * unit          # every group before gb is done
                far_so = so[new & valid]
                assert (far_so + 128 <= flushed).all()
