"""Nothing is written outside a value's output range (needs a GPU).

Every value's output region out[out_off, out_off + out_cap) is followed by a
guard gap; the arena starts as a canary pattern.  After compress (server
caps, tight caps, failing caps) and decompress (valid, E2BIG, EINVAL
streams) every guard byte is unchanged.  A batch whose stated max length is
below a value's length (a caller contract violation) refuses that value --
out_len 0 (and EINVAL on decompress) -- and leaves its region untouched
(include/lzf_gpu.h)."""
import random

import numpy as np
import pytest

from tests.oracle_lib import synth

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

CANARY = 0xA5
GUARD = 64


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture(autouse=True)
def _lane_for_any_batch(monkeypatch):
    monkeypatch.setenv("LZF_GPU_LANE_MIN", "0")


def _layout(caps):
    offs, pos = [], 0
    for c in caps:
        offs.append(pos)
        pos += c + GUARD
    return np.array(offs, np.int64), pos


def _run_compress(vals, caps, max_len):
    import gibson_amd
    dev = "cuda"
    in_offs, pos = [], 0
    for v in vals:
        in_offs.append(pos)
        pos += len(v) + 7
    arena = np.zeros(pos + 16, np.uint8)
    for o, v in zip(in_offs, vals):
        arena[o:o + len(v)] = np.frombuffer(v, np.uint8)
    out_off, size = _layout(caps)
    out = torch.full((size,), CANARY, dtype=torch.uint8, device=dev)
    olen = torch.full((len(vals),), 0x7777, dtype=torch.int32, device=dev)
    gibson_amd.compress_batch(torch.from_numpy(arena).to(dev), torch.tensor(in_offs, device=dev),
                              torch.tensor([len(v) for v in vals], dtype=torch.int32, device=dev), out,
                              torch.from_numpy(out_off).to(dev), torch.tensor(caps, dtype=torch.int32, device=dev),
                              olen, max_len)
    torch.cuda.synchronize()
    return out.cpu().numpy(), out_off, olen.cpu().numpy()


def _guards_intact(out, offs, caps):
    for o, c in zip(offs, caps):
        g = out[o + c:o + c + GUARD]
        if not (g == CANARY).all():
            return False
    return True


@pytest.mark.parametrize("nmax", [4096, 16384, 65536])
def test_compress_writes_nothing_past_out_cap(oracle, nmax):
    rnd = random.Random(nmax)
    vals, caps = [], []
    for i in range(400):
        n = rnd.randint(1, nmax)
        v = synth(rnd.randrange(6), 0x5EED0B00, i, n)
        full = oracle.compress(v, n + n // 16 + 64)
        F = len(full) if full else n
        caps.append(max(1, rnd.choice([n - 4, F - 1, F, F + 1, rnd.randint(1, n + 8), F // 2])))
        vals.append(v)
    out, offs, olen = _run_compress(vals, caps, nmax)
    assert _guards_intact(out, offs, caps)
    for v, c, o, ln in zip(vals, caps, offs, olen):
        exp = oracle.compress(v, c)
        assert (bytes(out[o:o + ln]) if ln else None) == exp


@pytest.mark.parametrize("nmax", [4096, 16384, 65536])
def test_free_literal_runs_at_tight_caps(oracle, nmax):
    # whole waves of random and mixed-entropy values, so the parses'
    # free-literal path (profiles/r03/INDEX.md: at least 8 lanes of a wave at a
    # literal with no candidate) runs, and caps that run out inside such runs
    rnd = random.Random(100 + nmax)
    vals, caps = [], []
    for i in range(320):
        n = rnd.choice([nmax, rnd.randint(nmax // 2, nmax)])
        kind = 4 if i % 3 else 3                       # random bytes, mixed entropy
        v = synth(kind, 0x5EED0B30, i, n)
        full = oracle.compress(v, n + n // 16 + 64)
        F = len(full) if full else n
        caps.append(max(1, rnd.choice([n - 4, F - 1, F, F + 33, rnd.randint(1, n), n // 3])))
        vals.append(v)
    out, offs, olen = _run_compress(vals, caps, nmax)
    assert _guards_intact(out, offs, caps)
    for v, c, o, ln in zip(vals, caps, offs, olen):
        assert (bytes(out[o:o + ln]) if ln else None) == oracle.compress(v, c)


def test_compress_refuses_value_past_stated_max_len(oracle):
    rnd = random.Random(3)
    vals = [synth(rnd.randrange(4), 0x5EED0B10, i, rnd.choice([900, 5000, 9000, 30000])) for i in range(200)]
    caps = [len(v) - 4 for v in vals]
    stated = 6000                       # below the 9000 / 30000 values
    out, offs, olen = _run_compress(vals, caps, stated)
    for v, c, o, ln in zip(vals, caps, offs, olen):
        if len(v) > stated:
            assert ln == 0
            assert (out[o:o + c + GUARD] == CANARY).all()
        else:
            assert (bytes(out[o:o + ln]) if ln else None) == oracle.compress(v, c)


def _run_decompress(streams, caps, max_cap):
    import gibson_amd
    dev = "cuda"
    in_offs, pos = [], 0
    for s in streams:
        in_offs.append(pos)
        pos += max(len(s), 1) + 5
    arena = np.full(pos + 16, 0xFF, np.uint8)
    for o, s in zip(in_offs, streams):
        arena[o:o + len(s)] = np.frombuffer(s, np.uint8)
    out_off, size = _layout(caps)
    out = torch.full((size,), CANARY, dtype=torch.uint8, device=dev)
    olen = torch.full((len(streams),), 0x7777, dtype=torch.int32, device=dev)
    err = torch.full((len(streams),), -1, dtype=torch.int32, device=dev)
    gibson_amd.decompress_batch(torch.from_numpy(arena).to(dev), torch.tensor(in_offs, device=dev),
                                torch.tensor([len(s) for s in streams], dtype=torch.int32, device=dev), out,
                                torch.from_numpy(out_off).to(dev), torch.tensor(caps, dtype=torch.int32, device=dev),
                                olen, err, max_cap)
    torch.cuda.synchronize()
    return out.cpu().numpy(), out_off, olen.cpu().numpy(), err.cpu().numpy()


def test_decompress_writes_nothing_past_out_cap(oracle):
    rnd = random.Random(17)
    streams, caps = [], []
    for i in range(500):
        n = rnd.randint(1, 20000)
        v = synth(rnd.randrange(6), 0x5EED0B20, i, n)
        s = oracle.compress(v, n + n // 16 + 64)
        kind = rnd.randrange(4)
        if kind == 1:
            s = s[:rnd.randrange(1, len(s))]                     # EINVAL (truncated)
        elif kind == 2:
            b = bytearray(s)
            b[rnd.randrange(len(b))] = rnd.randrange(256)       # corrupted
            s = bytes(b)
        cap = n if kind != 3 else rnd.randint(1, max(1, n - 1))  # E2BIG
        streams.append(s)
        caps.append(cap)
    out, offs, olen, err = _run_decompress(streams, caps, 20000)
    assert _guards_intact(out, offs, caps)
    for s, c, o, ln, e in zip(streams, caps, offs, olen, err):
        exp, ee = oracle.decompress(s, c)
        assert (bytes(out[o:o + ln]) if ln else None, int(e)) == (exp, ee)


def test_decompress_refuses_cap_past_stated_max(oracle):
    import errno
    vals = [synth(0, 0x5EED0B30, i, 3000 + 1000 * (i % 8)) for i in range(64)]
    streams = [oracle.compress(v, len(v) + 64) for v in vals]
    caps = [len(v) for v in vals]
    stated = 6500
    out, offs, olen, err = _run_decompress(streams, caps, stated)
    for v, c, o, ln, e in zip(vals, caps, offs, olen, err):
        if c > stated:
            assert ln == 0 and e == errno.EINVAL
            assert (out[o:o + c + GUARD] == CANARY).all()
        else:
            assert bytes(out[o:o + ln]) == v and e == 0
