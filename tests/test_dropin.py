"""The single-call drop-in (include/lzf.h) as Gibson's callers use it (needs
a GPU): a C99 program linked against liblzf_hip.so replays the known answers,
GET/MGET decompress at the server's out_len (maxrequestsize: 4 MiB default,
src/default.h:45; 2 MiB in debian/etc/gibson/gibson.conf:29; passed at
src/net.c:1229-1235 and :1309), the single-call latency, and the failure
policy when no device is usable."""
import os
import random
import subprocess
import sys
import time

import pytest

from tests.oracle_lib import ROOT, synth

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

MAXREQ = (4 << 20, 2 << 20)
KAT_BIN = os.path.join(ROOT, "tests", "c", "kat_replay")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _server_streams(oracle):
    """Streams an LZF item can hold: SET-compressed values (out_len = n-4,
    src/query.c:385), plus truncated / corrupted ones for errno parity."""
    rnd = random.Random(45)
    out = []
    for i in range(120):
        n = rnd.choice([4097, 8192, 16384, 65536, rnd.randint(5, 70000)])
        v = synth(rnd.randrange(4), 0x5EED0D00, i, n)
        s = oracle.compress(v, n - 4)
        if not s:
            continue
        out.append(s)
        cut = s[:rnd.randrange(1, len(s))]
        out.append(cut)
        bad = bytearray(s)
        for _ in range(3):
            bad[rnd.randrange(len(bad))] = rnd.randrange(256)
        out.append(bytes(bad))
    return out


def _hx(b):
    return b.hex() if b else "-"


def test_c99_caller_replays_known_answers(kat, golden, oracle):
    from tests.test_oracle import decoder_cases
    assert os.path.exists(KAT_BIN), "tests/c/kat_replay not built (__graft_entry__.build())"
    lines = []
    for c in kat:
        if c["op"] == "compress":
            lines.append(f"C {_hx(bytes.fromhex(c['in_hex']))} {c['out_len']} {c['result']} {c['out_hex'] or '-'}")
        else:
            lines.append(f"D {_hx(bytes.fromhex(c['in_hex']))} {c['out_len']} {c['result']} {c['errno']} "
                         f"{c['out_hex'] or '-'}")
    # decoder cases of the golden corpus at their own out_len and at maxrequestsize
    for c, s in list(decoder_cases(golden, oracle))[:400]:
        if not s:
            continue
        for cap in (c["out_len"], MAXREQ[0]):
            out, e = oracle.decompress(s, cap)
            lines.append(f"D {_hx(s)} {cap} {len(out) if out else 0} {e} {_hx(out)}")
    r = subprocess.run([KAT_BIN], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-500:] + r.stderr[-500:]
    assert r.stdout.startswith("ok ")


@pytest.mark.parametrize("cap", MAXREQ)
def test_decompress_at_maxrequestsize(oracle, cap):
    import gibson_amd
    for s in _server_streams(oracle):
        assert gibson_amd.lzf_decompress(s, cap) == oracle.decompress(s, cap)


def test_single_call_latency_recorded(oracle):
    """Every SET/GET through the drop-in pays one H2D + launch + D2H + sync;
    the figures are recorded in DESIGN.md §5 (printed here with -s)."""
    import gibson_amd
    res = {}
    for n in (4096, 65536):
        v = synth(2, 0x5EED0003, 7, n)
        s = gibson_amd.lzf_compress(v, n - 4)
        assert s == oracle.compress(v, n - 4)
        for op in ("compress", "decompress"):
            f = (lambda: gibson_amd.lzf_compress(v, n - 4)) if op == "compress" else \
                (lambda: gibson_amd.lzf_decompress(s, MAXREQ[0]))
            for _ in range(20):
                f()
            t = []
            for _ in range(200):
                t0 = time.perf_counter()
                f()
                t.append(time.perf_counter() - t0)
            t.sort()
            res[(op, n)] = t[len(t) // 2] * 1e6
    print("single-call median us:", {f"{k[0]} {k[1]}": round(u, 1) for k, u in res.items()})
    assert all(u < 20000 for u in res.values())


def _config0():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "config0.json")) as f:
        return json.load(f)


def test_config0_roundtrip_dropin():
    """BASELINE configs[0] by its own generator: the 64 KiB text value at seed
    0x5EED0001 through the drop-in lzf_compress (out_len = n-4,
    src/query.c:385) and lzf_decompress (out_len = maxrequestsize,
    src/net.c:1234): the stream is the reference's (tests/golden/config0.json,
    from oracle/_ref) and decodes to the value."""
    import hashlib
    import gibson_amd
    c = _config0()
    v = synth(c["kind"], c["seed"], c["index"], c["n"])
    assert hashlib.sha256(v).hexdigest() == c["in_sha256"]
    s = gibson_amd.lzf_compress(v, c["out_len"])
    assert s is not None and len(s) == c["stream_len"]
    assert hashlib.sha256(s).hexdigest() == c["stream_sha256"]
    out, e = gibson_amd.lzf_decompress(s, c["decode_out_len"])
    assert (len(out), e) == (c["decode_result"], c["decode_errno"]) and out == v


def test_release_then_reuse(oracle):
    import gibson_amd
    from tests.gpu_batch import gpu_compress
    vals = [synth(k % 6, 0x5EED0E00, k, 9000 + 37 * k) for k in range(50)]
    caps = [len(v) - 4 for v in vals]
    a = gpu_compress(vals, caps)
    gibson_amd.release()
    assert gpu_compress(vals, caps) == a == [oracle.compress(v, c) for v, c in zip(vals, caps)]
    v = synth(1, 3, 3, 5000)
    assert gibson_amd.lzf_compress(v, 4996) == oracle.compress(v, 4996)
    gibson_amd.release()
    assert gibson_amd.lzf_decompress(oracle.compress(v, 4996), MAXREQ[0]) == (v, 0)


def test_no_usable_device_is_reported_not_aborted():
    # a device index past the machine's: the drop-in never aborts the server
    code = ("import ctypes, errno, sys; sys.path.insert(0, %r); import gibson_amd as g; "
            "print(g.lzf_compress(b'abcabcabcabcabc' * 10, 140), g.lzf_decompress(b'\\x00a', 10))" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, LZF_GPU_DEVICE="97"))
    assert r.returncode == 0, r.stderr[-500:]
    import errno
    assert r.stdout.strip() == f"None (None, {errno.EIO})", r.stdout
