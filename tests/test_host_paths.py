"""The host-memory batch calls on the GPU: registered arenas (no CPU byte
copies, lzf_host_register) against the staged path and the oracle, and the
multi-device plan (LZF_GPU_DEVICES) inside the library -- value i to plan
entry i mod G, each entry a worker thread with its own streams and staging --
run as two contexts on the box's one device ("0,0"), bit-exact against the
oracle and the reference's configs[1] digest."""
import json
import os
import random
import subprocess
import sys

import numpy as np
import pytest

from tests.oracle_lib import ROOT, synth

pytestmark = pytest.mark.gpu


def _aligned(nbytes):
    raw = np.zeros(nbytes + 8192, np.uint8)
    k = (-raw.ctypes.data) % 4096
    return raw[k:k + nbytes]


@pytest.fixture
def registered():
    import gibson_amd
    held = []

    def reg(a):
        gibson_amd.host_register(a)
        held.append(a)
        return a
    yield reg
    for a in held:
        gibson_amd.host_unregister(a)


def test_registered_matches_staged_and_oracle(oracle, registered):
    # shuffled, unaligned arena order with mixed sizes (0 B .. 20 KiB): the
    # GPU gathers the values from the mapped arena and scatters the streams
    import gibson_amd
    rnd = random.Random(31)
    count = 6000
    sizes = [rnd.choice([4096, 4096, rnd.randint(0, 20000)]) for _ in range(count)]
    order = list(range(count))
    rnd.shuffle(order)
    pos, offs = 0, [0] * count
    for i in order:
        offs[i] = pos
        pos += sizes[i] + rnd.randint(0, 3)
    arena = registered(_aligned(pos + 16))
    for i in range(count):
        arena[offs[i]:offs[i] + sizes[i]] = np.frombuffer(synth(i % 6, 0x5EED00B1, i, sizes[i]), np.uint8)
    off = np.array(offs, dtype=np.uint64)
    ln = np.array(sizes, dtype=np.uint32)
    cap = np.maximum(ln.astype(np.int64) - 4, 0).astype(np.uint32)
    out_r = registered(_aligned(pos + 16))
    olen_r = np.zeros(count, np.uint32)
    gibson_amd.host_compress_batch(arena, off, ln, out_r, off, cap, olen_r)
    # the same batch staged (an unregistered output arena)
    out_s = np.zeros(pos + 16, np.uint8)
    olen_s = np.zeros(count, np.uint32)
    gibson_amd.host_compress_batch(arena, off, ln, out_s, off, cap, olen_s)
    assert np.array_equal(olen_r, olen_s)
    for i in range(count):
        got = bytes(out_r[offs[i]:offs[i] + olen_r[i]]) if olen_r[i] else None
        assert got == (bytes(out_s[offs[i]:offs[i] + olen_s[i]]) if olen_s[i] else None), i
    for i in rnd.sample(range(count), 600):
        v = bytes(arena[offs[i]:offs[i] + sizes[i]])
        exp = oracle.compress(v, int(cap[i])) if sizes[i] and cap[i] else None
        got = bytes(out_r[offs[i]:offs[i] + olen_r[i]]) if olen_r[i] else None
        assert got == exp, i
    ok = olen_r > 0
    dec = registered(_aligned(pos + 16))
    dl = np.zeros(int(ok.sum()), np.uint32)
    er = np.zeros(int(ok.sum()), np.int32)
    gibson_amd.host_decompress_batch(out_r, off[ok], olen_r[ok], dec, off[ok], ln[ok], dl, er)
    assert (dl == ln[ok]).all() and (er == 0).all()
    for i in np.nonzero(ok)[0]:
        assert bytes(dec[offs[i]:offs[i] + sizes[i]]) == bytes(arena[offs[i]:offs[i] + sizes[i]]), i


def test_registered_contiguous_runs_and_exact_writes(oracle, registered):
    # values back to back (the DMA engines copy whole runs) and output slots
    # with guard bytes between them: the scatter writes exactly out_len bytes
    import gibson_amd
    count, n = 4096, 4096
    arena = registered(_aligned(count * n))
    for i in range(count):
        arena[i * n:(i + 1) * n] = np.frombuffer(synth(i % 6, 0x5EED00B2, i, n), np.uint8)
    off = np.arange(count, dtype=np.uint64) * n
    ln = np.full(count, n, np.uint32)
    cap = np.full(count, n - 4, np.uint32)
    slot = n + 64
    out = registered(_aligned(count * slot))
    out[:] = 0xA5
    oof = np.arange(count, dtype=np.uint64) * slot
    olen = np.zeros(count, np.uint32)
    gibson_amd.host_compress_batch(arena, off, ln, out, oof, cap, olen)
    for i in range(count):
        s = out[i * slot:(i + 1) * slot]
        exp = oracle.compress(bytes(arena[i * n:(i + 1) * n]), n - 4)
        if exp is None:
            assert olen[i] == 0
        else:
            assert bytes(s[:olen[i]]) == exp, i
            assert (s[olen[i]:] == 0xA5).all(), i
    # decoded values into abutting slots: the DMA engines write whole runs
    ok = olen > 0
    dec = registered(_aligned(count * n))
    dl = np.zeros(int(ok.sum()), np.uint32)
    er = np.zeros(int(ok.sum()), np.int32)
    m = int(ok.sum())
    gibson_amd.host_decompress_batch(out, oof[ok], olen[ok], dec, np.arange(m, dtype=np.uint64) * n,
                                     np.full(m, n, np.uint32), dl, er)
    assert (dl == n).all() and (er == 0).all()
    assert np.array_equal(dec[:m * n].reshape(m, n), arena.reshape(count, n)[ok])


def test_registered_decode_errors_and_empty_streams(oracle, registered):
    # decoder errno parity through the registered path: truncated and
    # corrupted streams, and 0-length streams (which read one control byte)
    import gibson_amd
    rnd = random.Random(5)
    streams, caps, exp = [], [], []
    for k in range(300):
        v = synth(k % 6, 0x5EED00B3, k, rnd.randint(1, 9000))
        s = oracle.compress(v, len(v) + len(v) // 16 + 64)
        if k % 3 == 1:
            s = s[:rnd.randint(0, len(s))]
        elif k % 3 == 2:
            b = bytearray(s)
            b[rnd.randrange(len(b))] ^= 0xFF
            s = bytes(b)
        c = len(v) if k % 5 else len(v) // 2
        streams.append(s)
        caps.append(c)
        exp.append(oracle.decompress(s, c))
    pos, offs = 0, []
    for s in streams:
        offs.append(pos)
        pos += len(s) + 1
    inp = registered(_aligned(pos + 16))
    for s, o in zip(streams, offs):
        inp[o:o + len(s)] = np.frombuffer(s, np.uint8)
        inp[o + len(s)] = 0xFF
    doff, p = [], 0
    for c in caps:
        doff.append(p)
        p += c + 7
    out = registered(_aligned(p + 16))
    dl = np.zeros(len(streams), np.uint32)
    er = np.zeros(len(streams), np.int32)
    gibson_amd.host_decompress_batch(inp, np.array(offs, np.uint64), np.array([len(s) for s in streams], np.uint32),
                                     out, np.array(doff, np.uint64), np.array(caps, np.uint32), dl, er)
    for k, (d, e) in enumerate(exp):
        if d is None:
            assert dl[k] == 0 and er[k] == e, k
        else:
            assert er[k] == 0 and bytes(out[doff[k]:doff[k] + dl[k]]) == d, k


def test_register_rejects_overlap():
    import gibson_amd
    a = _aligned(1 << 20)
    gibson_amd.host_register(a)
    try:
        with pytest.raises(RuntimeError):
            gibson_amd.host_register(a[4096:8192])
    finally:
        gibson_amd.host_unregister(a)


@pytest.mark.parametrize("split", ["rr", "block"])
def test_two_contexts_on_one_device_bit_exact(digests_full, split):
    # LZF_GPU_DEVICES=0,0: the round-robin split (default) or the contiguous
    # one (LZF_GPU_SPLIT=block) over two worker contexts, staged and
    # registered, against the oracle and configs[1]'s digest
    env = dict(os.environ, LZF_GPU_DEVICES="0,0", LZF_GPU_SPLIT=split)
    env.pop("LZF_GPU_LANE_MIN", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "host_devices_run.py")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert [p[0] for p in res["plan"]] == [0, 0]
    assert res["split"] == ("block" if split == "block" else "round-robin")
    want = digests_full[(1, 0x5EED0002, 4096, 262144)]
    for tag in ("staged", "registered"):
        m = res["mixed_" + tag]
        assert m["mismatches"] == 0 and m["roundtrip"], (tag, m)
        assert [s[0] for s in m["spread"]] == [1500, 1500], m["spread"]
        c = res["config1_" + tag]
        assert c["digest"] == want, tag
        assert [s[0] for s in c["spread"]] == [131072, 131072]


@pytest.fixture(scope="module")
def digests_full():
    with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
        return {(d["kind"], d["seed"], d["n"], d["count"]): d["sha256"] for d in json.load(f)["digests"]
                if not d.get("first")}


def test_registered_bulk_chunks_config1_digest(digests_full, registered):
    # 1 GiB of configs[1] through registered arenas: three side-by-side
    # chunks on the slots' own scratch (the bulk route), bit-exact by the
    # reference's digest of the first 262 144 values
    import gibson_amd
    from tests.digest import batch_digest
    from tests.oracle_lib import _SYN
    kind, seed, n, count = 1, 0x5EED0002, 4096, 262144
    arena = registered(_aligned(count * n))
    _SYN.synth_fill(kind, seed, 0, count, n, arena.ctypes.data)
    off = np.arange(count, dtype=np.uint64) * n
    out = registered(_aligned(count * n))
    olen = np.zeros(count, np.uint32)
    gibson_amd.host_compress_batch(arena, off, np.full(count, n, np.uint32), out, off,
                                   np.full(count, n - 4, np.uint32), olen)
    assert batch_digest(out, n, olen) == digests_full[(kind, seed, n, count)]


def test_bad_device_plan_is_reported_not_aborted():
    # an LZF_GPU_DEVICES entry past the machine's devices: every host call
    # returns LZF_GPU_ENODEV (the plan is read once, in a child process)
    code = ("import numpy as np, gibson_amd\n"
            "a = np.zeros(8192, np.uint8); o = np.zeros(8192, np.uint8)\n"
            "off = np.zeros(1, np.uint64); ln = np.full(1, 8192, np.uint32); cap = np.full(1, 8188, np.uint32)\n"
            "ol = np.zeros(1, np.uint32)\n"
            "L = gibson_amd.lib()\n"
            "p = lambda x: x.ctypes.data\n"
            "print(L.lzf_host_compress_batch(p(a), p(off), p(ln), p(o), p(off), p(cap), p(ol), 1))\n"
            "print(L.lzf_gpu_device_plan(None, None, None, 0))\n")
    env = dict(os.environ, LZF_GPU_DEVICES="0,63")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.split() == ["-3", "-3"], r.stdout


@pytest.mark.parametrize("share,chunks,cap_mb,scratch_mb",
                         [(None, None, None, None), (50, 4, None, None), (None, None, 64, None), (None, None, 24, None),
                          (None, None, None, 1140), (None, None, None, 1024)],
                         ids=["default", "50pct-4chunks", "cap64MiB", "cap24MiB-slot-reuse",
                              "scratch-table-2chunks", "scratch-lane"])
def test_registered_tail_mode_64k(oracle, registered, monkeypatch, share, chunks, cap_mb, scratch_mb):
    # 256 MiB of 64 KiB values (configs[2]'s generator): the registered path's
    # tail mode -- the first part of the values through the table generation,
    # the rest by window64 in chunks beside its parse (default 70 % and one
    # chunk; 50 % and four, each chunk in its own slot; under a chunk cap
    # (LZF_GPU_HOST_CHUNK_MB) both parts split into chunks of at most the cap:
    # 64 MiB gives 3 + 2 chunks, 24 MiB 8 + 4, more chunks than slots) --
    # against the staged path and a sample of the oracle that includes every
    # chunk boundary
    if share is not None:
        monkeypatch.setenv("LZF_GPU_HOST_TAIL", str(share))
        monkeypatch.setenv("LZF_GPU_HOST_TAIL_CHUNKS", str(chunks))
    if cap_mb is not None:
        monkeypatch.setenv("LZF_GPU_HOST_CHUNK_MB", str(cap_mb))
    if scratch_mb is not None:
        # a scratch cap (each of the three slots holds a third): the routed
        # chunk's cand parts then meet a table generation in two scratch
        # chunks (1140 MiB) or the lane generation (1024 MiB), both of which
        # wait for every input part before their first kernel
        monkeypatch.setenv("LZF_GPU_SCRATCH_MB", str(scratch_mb))
    import gibson_amd
    from tests.oracle_lib import _SYN
    n, count = 65536, 4096
    arena = registered(_aligned(count * n))
    _SYN.synth_fill(2, 0x5EED0003, 0, count, n, arena.ctypes.data)
    off = np.arange(count, dtype=np.uint64) * n
    ln = np.full(count, n, np.uint32)
    cap = np.full(count, n - 4, np.uint32)
    out_r = registered(_aligned(count * n))
    olen_r = np.zeros(count, np.uint32)
    gibson_amd.host_compress_batch(arena, off, ln, out_r, off, cap, olen_r)
    out_s = np.zeros(count * n, np.uint8)
    olen_s = np.zeros(count, np.uint32)
    gibson_amd.host_compress_batch(arena, off, ln, out_s, off, cap, olen_s)
    assert np.array_equal(olen_r, olen_s)
    for i in range(count):
        assert np.array_equal(out_r[i * n:i * n + olen_r[i]], out_s[i * n:i * n + olen_s[i]]), i
    pct, nch = (share or 70), (chunks or 1)
    t = count * pct // 100
    edges = [t + (count - t) * k // nch for k in range(nch)]
    if cap_mb is not None:                       # the capped plan's chunk edges (equal bytes: equal counts here)
        per = (cap_mb << 20) // n
        r = -(-t // per)
        q = max(nch, -(-(count - t) // per))
        edges += [t * k // r for k in range(r)] + [t + (count - t) * k // q for k in range(q)]
    for i in sorted({i for i in list(range(0, count, 97)) + [e + d for e in edges for d in (-1, 0)] + [count - 1]
                     if 0 <= i < count}):
        exp = oracle.compress(bytes(arena[i * n:(i + 1) * n]), n - 4)
        assert bytes(out_r[i * n:i * n + olen_r[i]]) == exp, i


@pytest.mark.parametrize("env", [{}, {"LZF_GPU_HOST_NCHUNKS": "1"}, {"LZF_GPU_HOST_TAIL": "0"},
                                 {"LZF_GPU_HOST_TAIL_CHUNKS": "3", "LZF_GPU_HOST_TAIL": "40"}],
                         ids=["default", "one-chunk", "tail-off", "tail40-3chunks"])
def test_registered_bulk_mixed_sizes(oracle, registered, monkeypatch, env):
    # a bulk compress batch (>= 192 MiB) of 0 B .. 64 KiB values at unaligned,
    # shuffled arena offsets: the chunk plan, the tail mode and its window64
    # part over ragged values, against the staged path and an oracle sample
    # that includes every chunk's edges; then the round trip
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    import gibson_amd
    rnd = random.Random(57)
    count = 12288
    sizes = [rnd.choice([65536, rnd.randint(0, 65536), rnd.randint(0, 20000)]) for _ in range(count)]
    order = list(range(count))
    rnd.shuffle(order)
    pos, offs = 0, [0] * count
    for i in order:
        offs[i] = pos
        pos += sizes[i] + rnd.randint(0, 5)
    assert pos >= 192 << 20
    arena = registered(_aligned(pos + 16))
    for i in range(count):
        arena[offs[i]:offs[i] + sizes[i]] = np.frombuffer(synth((2, 3, 1)[i % 3], 0x5EED00B5, i, sizes[i]), np.uint8)
    off = np.array(offs, dtype=np.uint64)
    ln = np.array(sizes, dtype=np.uint32)
    cap = np.maximum(ln.astype(np.int64) - 4, 0).astype(np.uint32)
    out_r = registered(_aligned(pos + 16))
    olen_r = np.zeros(count, np.uint32)
    gibson_amd.host_compress_batch(arena, off, ln, out_r, off, cap, olen_r)
    out_s = np.zeros(pos + 16, np.uint8)
    olen_s = np.zeros(count, np.uint32)
    gibson_amd.host_compress_batch(arena, off, ln, out_s, off, cap, olen_s)
    assert np.array_equal(olen_r, olen_s)
    for i in range(count):
        assert bytes(out_r[offs[i]:offs[i] + olen_r[i]]) == bytes(out_s[offs[i]:offs[i] + olen_s[i]]), i
    edges = {0, count - 1} | {count * p // 100 + d for p in (40, 70) for d in (-1, 0)} | \
        {count * k // 3 + d for k in (1, 2) for d in (-1, 0)}
    for i in sorted(edges | set(rnd.sample(range(count), 150))):
        v = bytes(arena[offs[i]:offs[i] + sizes[i]])
        exp = oracle.compress(v, int(cap[i])) if sizes[i] and cap[i] else None
        got = bytes(out_r[offs[i]:offs[i] + olen_r[i]]) if olen_r[i] else None
        assert got == exp, i
    ok = olen_r > 0
    dec = registered(_aligned(pos + 16))
    dl = np.zeros(int(ok.sum()), np.uint32)
    er = np.zeros(int(ok.sum()), np.int32)
    gibson_amd.host_decompress_batch(out_r, off[ok], olen_r[ok], dec, off[ok], ln[ok], dl, er)
    assert (dl == ln[ok]).all() and (er == 0).all()
    for i in np.nonzero(ok)[0]:
        assert bytes(dec[offs[i]:offs[i] + sizes[i]]) == bytes(arena[offs[i]:offs[i] + sizes[i]]), i


def test_register_refused_unless_every_plan_device_maps(monkeypatch):
    # lzf_host_register asks every distinct device of the plan for the
    # range's device address (first and last byte); a device that gives none
    # (forced here for device 0) makes the registration fail whole: ENODEV,
    # the range left unregistered, and it registers normally afterwards
    import gibson_amd
    a = _aligned(1 << 20)
    monkeypatch.setenv("LZF_GPU_FORCE_MAP_FAIL", "0")
    with pytest.raises(RuntimeError, match="ENODEV"):
        gibson_amd.host_register(a)
    monkeypatch.delenv("LZF_GPU_FORCE_MAP_FAIL")
    gibson_amd.host_register(a)
    gibson_amd.host_unregister(a)


@pytest.mark.parametrize("dchunk_mb,gapped", [(None, False), ("1", False), (None, True)],
                         ids=["abutting-dma", "abutting-dma-chunks", "gapped-scatter"])
def test_registered_decode_leaves_no_stale_bytes(oracle, registered, monkeypatch, dchunk_mb, gapped):
    # abutting output slots go back to the caller as DMA runs of whole slots:
    # a second batch into the same layout whose streams decode short or fail
    # must not carry the first batch's decoded bytes past its own out_len
    # (they are zeroed on the device first); also with 1 MiB decode chunks
    if dchunk_mb:
        monkeypatch.setenv("LZF_GPU_HOST_DCHUNK_MB", dchunk_mb)
    import gibson_amd
    count, n = 512, 4096
    vals = [synth(k % 6, 0x5EED00B7, k, n) for k in range(count)]
    streams = [oracle.compress(v, n + n // 16 + 64) for v in vals]   # every value fits (incompressible ones grow)
    pos, offs = 0, []
    for st in streams:
        offs.append(pos)
        pos += len(st)
    inp = registered(_aligned(pos + 16))
    for st, o in zip(streams, offs):
        inp[o:o + len(st)] = np.frombuffer(st, np.uint8)
    out = registered(_aligned(count * n))
    doff = np.arange(count, dtype=np.uint64) * n
    dl = np.zeros(count, np.uint32)
    er = np.zeros(count, np.int32)
    ioff = np.array(offs, np.uint64)
    ilen = np.array([len(st) for st in streams], np.uint32)
    gibson_amd.host_decompress_batch(inp, ioff, ilen, out, doff, np.full(count, n, np.uint32), dl, er)
    assert (dl == n).all() and bytes(out[:n]) == vals[0]
    # the same slots again, every third stream truncated (it fails, or ends
    # early at a token boundary). Abutting slots go back as one DMA run of
    # whole slots: the bytes past each out_len must be zeros, not the first
    # batch's decoded bytes still in the device arena. Gapped slots (every
    # third cap halved, E2BIG for some) go back by the scatter kernel, which
    # writes exactly out_len bytes: the caller's own bytes stay.
    cut = ilen.copy()
    cut[0::3] = np.maximum(cut[0::3] // 2, 1)
    caps = np.full(count, n, np.uint32)
    if gapped:
        caps[1::3] = n // 2
    out[:] = 0xA5
    gibson_amd.host_decompress_batch(inp, ioff, cut, out, doff, caps, dl, er)
    short = 0
    for k in range(count):
        e = oracle.decompress(bytes(inp[offs[k]:offs[k] + cut[k]]), int(caps[k]))
        s = out[k * n:(k + 1) * n]
        if e[0] is None:
            assert dl[k] == 0 and er[k] == e[1], k
        else:
            assert bytes(s[:dl[k]]) == e[0], k
        tail = s[dl[k]:caps[k]]
        short += tail.size > 0
        assert (tail == (0xA5 if gapped else 0)).all(), k    # no stale device bytes
    assert short > count // 4


def test_worker_plan_made_whole_or_not_at_all():
    # LZF_GPU_DEVICES=0,0 with the second worker's creation failing
    # (LZF_GPU_FORCE_WORKER_FAIL=1): the call returns LZF_GPU_ENOMEM and
    # nothing runs on a partial plan; with the failure gone, the next call
    # completes the plan and the batch is bit-exact against the oracle
    code = ("import os, numpy as np, gibson_amd\n"
            "from tests.oracle_lib import Oracle, synth\n"
            "n, count = 4096, 64\n"
            "a = np.frombuffer(b''.join(synth(k % 6, 0x5EED00B9, k, n) for k in range(count)), np.uint8).copy()\n"
            "o = np.zeros(count * n, np.uint8); off = np.arange(count, dtype=np.uint64) * n\n"
            "ln = np.full(count, n, np.uint32); cap = np.full(count, n - 4, np.uint32); ol = np.zeros(count, np.uint32)\n"
            "L = gibson_amd.lib(); p = lambda x: x.ctypes.data\n"
            "print(L.lzf_host_compress_batch(p(a), p(off), p(ln), p(o), p(off), p(cap), p(ol), count))\n"
            "print(L.lzf_gpu_device_plan(None, None, None, 0))\n"
            "del os.environ['LZF_GPU_FORCE_WORKER_FAIL']\n"
            "print(L.lzf_host_compress_batch(p(a), p(off), p(ln), p(o), p(off), p(cap), p(ol), count))\n"
            "print(L.lzf_gpu_device_plan(None, None, None, 0))\n"
            "orc = Oracle()\n"
            "bad = sum((bytes(o[k*n:k*n+ol[k]]) if ol[k] else None) != orc.compress(bytes(a[k*n:(k+1)*n]), n - 4)\n"
            "          for k in range(count))\n"
            "print(bad, [v for v, _ in gibson_amd.host_last_spread()])\n")
    env = dict(os.environ, LZF_GPU_DEVICES="0,0", LZF_GPU_FORCE_WORKER_FAIL="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    out = r.stdout.split("\n")
    assert out[0] == "-4" and out[1] == "-4", r.stdout           # ENOMEM: no partial plan runs
    assert out[2] == "0" and out[3] == "2", r.stdout
    assert out[4] == "0 [32, 32]", r.stdout
