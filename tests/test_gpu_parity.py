"""Parity of the HIP path with the oracle / golden vectors (needs a GPU).

Everything here calls through the C-ABI of liblzf_hip.so: the drop-in pair
(include/lzf.h) and the device batch API (include/lzf_gpu.h).  The bar is
bit-exact: compressed streams, return values and errno are identical to the
reference's (pinned by tests/golden and tests/test_oracle.py).
"""
import contextlib
import errno
import os
import random

import numpy as np
import pytest

from tests.oracle_lib import sha16, synth

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

# "default": the library's routing (lane generation with the stream cand
# kernel up to 16 KiB, table generation to 64 KiB); the rest forced
GENERATIONS = ["default", "table", "table-stream", "wtab", "lane", "lane-small", "window", "serial", "lane-diag"]
# cross-check forms the product routing never takes: the diagnostic build only
DIAG = {"serial", "lane-diag", "wtab", "table-stream", "lane-small"}
GEN_ENV = {
    "default": {},
    "table": {"LZF_GPU_KERNEL": "table"},
    "table-stream": {"LZF_GPU_KERNEL": "table", "LZF_GPU_TCAND": "stream"},   # records from the stream kernel
    "wtab": {"LZF_GPU_KERNEL": "wtab"},
    "lane": {"LZF_GPU_KERNEL": "lane"},                              # stream cand kernel
    "lane-small": {"LZF_GPU_KERNEL": "lane", "LZF_GPU_CAND": "small"},  # small class (<= 4 KiB)
    "window": {"LZF_GPU_KERNEL": "window"},
    "serial": {"LZF_GPU_KERNEL": "serial"},
    "lane-diag": {"LZF_GPU_KERNEL": "lane", "LZF_GPU_CAND": "small"},   # diag: small/ring classes
}


@pytest.fixture(autouse=True)
def _lane_for_any_batch(monkeypatch):
    # the library routes batches below LZF_GPU_LANE_MIN values to the window
    # generation (faster there); the parity batches here are small, so the
    # lane kernels are asked for explicitly
    monkeypatch.setenv("LZF_GPU_LANE_MIN", "0")


@contextlib.contextmanager
def _diag():
    import gibson_amd
    path = gibson_amd.lzf.diag_lib_path()
    if not os.path.exists(path):
        pytest.skip("diagnostic build not present")
    with gibson_amd.lzf.using(path):
        yield


@pytest.fixture
def diag():
    with _diag():
        yield


@pytest.fixture(params=GENERATIONS)
def generation(request, monkeypatch):
    gen = request.param
    monkeypatch.delenv("LZF_GPU_KERNEL", raising=False)
    monkeypatch.delenv("LZF_GPU_CAND", raising=False)
    monkeypatch.delenv("LZF_GPU_TCAND", raising=False)
    for k, v in GEN_ENV[gen].items():
        monkeypatch.setenv(k, v)
    if gen in DIAG:
        with _diag():
            yield gen
    else:
        yield gen


def _limit(gen):
    # the serial generation keeps 16-bit positions
    import gibson_amd
    return 65536 if "compress=serial" in gibson_amd.kernel_info() else 1 << 30


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gibson_amd
    gibson_amd.lib()


def test_kernel_info_names_native_path():
    import gibson_amd
    info = gibson_amd.kernel_info()
    assert "compress=" in info and "decompress=" in info


def test_single_call_dropin_kat(kat):
    import gibson_amd
    for c in kat:
        data = bytes.fromhex(c["in_hex"])
        if c["op"] == "compress":
            r = gibson_amd.lzf_compress(data, c["out_len"])
            assert (len(r) if r else 0) == c["result"], c
            if r:
                assert r.hex() == c["out_hex"]
        else:
            out, e = gibson_amd.lzf_decompress(data, c["out_len"])
            assert (len(out) if out else 0) == c["result"], c
            assert e == c["errno"], c
            if out:
                assert out.hex() == c["out_hex"]


def test_batch_compress_golden(golden, generation):
    from tests.gpu_batch import gpu_compress
    cases = [c for c in golden["compress"] if c["n"] <= _limit(generation)]
    inputs = {}
    for c in cases:
        key = (c["kind"], c["seed"], c["index"], c["n"])
        if key not in inputs:
            inputs[key] = synth(*key)
    vals = [inputs[(c["kind"], c["seed"], c["index"], c["n"])] for c in cases]
    caps = [c["out_len"] for c in cases]
    res = gpu_compress(vals, caps)
    bad = []
    for c, r in zip(cases, res):
        if (len(r) if r else 0) != c["result"] or (r and sha16(r) != c["out_sha"]):
            bad.append((c["kind"], c["n"], c["out_len"], c["result"], len(r) if r else 0))
    assert not bad, f"{len(bad)} mismatches, first: {bad[:5]}"


@pytest.mark.parametrize("nmax", [4096, 8192, 16384, 65536])
def test_batch_compress_golden_by_size(golden, generation, nmax):
    # batches whose largest value selects each kernel class of a generation
    # (a batch with any value past 64 KiB runs the window generation)
    from tests.gpu_batch import gpu_compress
    cases = [c for c in golden["compress"] if c["n"] <= min(nmax, _limit(generation))]
    vals = [synth(c["kind"], c["seed"], c["index"], c["n"]) for c in cases]
    res = gpu_compress(vals, [c["out_len"] for c in cases])
    bad = [(c["kind"], c["n"], c["out_len"]) for c, r in zip(cases, res)
           if (len(r) if r else 0) != c["result"] or (r and sha16(r) != c["out_sha"])]
    assert not bad, f"{len(bad)} mismatches, first: {bad[:5]}"


def test_batch_decompress_golden(golden, oracle):
    from tests.gpu_batch import gpu_decompress
    from tests.test_oracle import decoder_cases
    cases = list(decoder_cases(golden, oracle))
    res = gpu_decompress([s for _, s in cases], [c["out_len"] for c, _ in cases])
    bad = []
    for (c, s), (out, e) in zip(cases, res):
        if (len(out) if out else 0) != c["result"] or e != c["errno"] or \
                (out and sha16(out) != c["out_sha"]):
            bad.append((c.get("tag"), c["n"] if "n" in c else None, c["result"], c["errno"],
                        len(out) if out else 0, e))
    assert not bad, f"{len(bad)} mismatches, first: {bad[:5]}"


def test_batch_decompress_golden_per_window(golden, oracle):
    # the decoder instance follows the batch's largest out_len (tokpar64 per
    # window of 256 B .. 4 KiB, the FAR route past that up to 16 KiB): the golden decoder
    # corpus (valid, tight, truncated, corrupted, random streams) split into
    # one batch per window size, so every instance meets the error cases
    from tests.gpu_batch import gpu_decompress
    from tests.test_oracle import decoder_cases
    buckets = {}
    for c, s in decoder_cases(golden, oracle):
        w = 256
        while w < c["out_len"] and w < 8192:
            w <<= 1
        buckets.setdefault(w, []).append((c, s))
    assert len(buckets) >= 4, sorted(buckets)
    for w, cases in sorted(buckets.items()):
        res = gpu_decompress([s for _, s in cases], [c["out_len"] for c, _ in cases])
        bad = [(c.get("tag"), c["result"], c["errno"], len(out) if out else 0, e)
               for (c, s), (out, e) in zip(cases, res)
               if (len(out) if out else 0) != c["result"] or e != c["errno"] or (out and sha16(out) != c["out_sha"])]
        assert not bad, f"window {w}: {len(bad)} mismatches of {len(cases)}, first: {bad[:5]}"


def test_batch_decompress_golden_on_pipe(golden, oracle):
    # the golden decoder corpus stops at 10 000-byte outputs, so its batches
    # take tokpar64 and the FAR route; one extra 20 000-byte value lifts the
    # batch's max_len past CD_FAR_MAX and every case through the pipe
    from tests.gpu_batch import gpu_decompress
    from tests.test_oracle import decoder_cases
    cases = list(decoder_cases(golden, oracle))
    extra = synth(2, 0x5EED0003, 7, 20000)
    xs = oracle.compress(extra, len(extra) + 64)
    res = gpu_decompress([s for _, s in cases] + [xs], [c["out_len"] for c, _ in cases] + [20000])
    assert res[-1] == (extra, 0)
    bad = [(c.get("tag"), c["result"], c["errno"], len(out) if out else 0, e)
           for (c, s), (out, e) in zip(cases, res)
           if (len(out) if out else 0) != c["result"] or e != c["errno"] or (out and sha16(out) != c["out_sha"])]
    assert not bad, f"{len(bad)} mismatches of {len(cases)}, first: {bad[:5]}"


def test_decoded_size_prepass_golden(golden, oracle):
    # the pre-pass (lzf_dsize.hip) against the reference's decode length and
    # errno on the whole golden decoder corpus: valid, tight, truncated at
    # every cut, corrupted and random streams
    import gibson_amd
    from tests.gpu_batch import _pack
    from tests.test_oracle import decoder_cases
    cases = list(decoder_cases(golden, oracle))
    streams = [s for _, s in cases]
    bad = []
    for limit in sorted({c["out_len"] for c, _ in cases}):
        sel = [(c, s) for c, s in cases if c["out_len"] == limit]
        arena, offs = _pack([s for _, s in sel])
        d_in = torch.from_numpy(arena).cuda()
        d_off = torch.from_numpy(offs).cuda()
        d_len = torch.tensor([len(s) for _, s in sel], dtype=torch.int32, device="cuda")
        size = torch.full((len(sel),), -1, dtype=torch.int32, device="cuda")
        err = torch.full((len(sel),), -1, dtype=torch.int32, device="cuda")
        gibson_amd.decoded_size_batch(d_in, d_off, d_len, size, err, limit)
        torch.cuda.synchronize()
        for (c, _), z, e in zip(sel, size.cpu().tolist(), err.cpu().tolist()):
            if z != c["result"] or e != c["errno"]:
                bad.append((c.get("tag"), limit, c["result"], c["errno"], z, e))
    assert streams and not bad, f"{len(bad)} mismatches, first: {bad[:5]}"


def test_lds_lane_order_selfcheck():
    # the probe the table / lane / window generations depend on
    # (lzf_selfcheck.hip), run as a library entry point; and the library's
    # one-time check is visible in kernel_info
    import gibson_amd
    assert gibson_amd.lds_order_probe() == 0
    assert gibson_amd.selfcheck() == 1
    assert "lds_order=held" in gibson_amd.kernel_info()


def test_lds_order_violation_falls_back_to_window64(golden, tmp_path):
    # a failed check routes compress batches to window64 (order-free): the
    # results stay bit-exact.  The check is per process, so in a child.
    import subprocess
    import sys
    code = (
        "import os, sys; sys.path.insert(0, %r)\n"
        "from tests.oracle_lib import synth, Oracle\n"
        "from tests.gpu_batch import gpu_compress\n"
        "import gibson_amd\n"
        "vals = [synth(k %% 4, 0x5EED0A30, k, 4096 * (1 + k %% 16)) for k in range(64)]\n"
        "caps = [len(v) - 4 for v in vals]\n"
        "o = Oracle()\n"
        "assert gpu_compress(vals, caps) == [o.compress(v, c) for v, c in zip(vals, caps)]\n"
        "assert gibson_amd.selfcheck() == 0\n"
        "info = gibson_amd.kernel_info()\n"
        "assert 'lds_order=violated' in info, info\n"
        "print('ok', info)\n") % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, LZF_GPU_FORCE_ORDER_FAIL="1", LZF_GPU_LANE_MIN="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("gen", ["window", "serial", "lane-decoder"])
def test_batch_decompress_other_generations(golden, oracle, monkeypatch, gen):
    if gen == "lane-decoder":
        monkeypatch.delenv("LZF_GPU_KERNEL", raising=False)
        monkeypatch.setenv("LZF_GPU_DECOMPRESS", "lane")
    else:
        monkeypatch.setenv("LZF_GPU_KERNEL", gen)
    if gen == "window":
        test_batch_decompress_golden(golden, oracle)
    else:
        with _diag():
            test_batch_decompress_golden(golden, oracle)


def test_lane_decoder_edge_and_unaligned(oracle, monkeypatch, diag):
    from tests.gpu_batch import gpu_decompress
    monkeypatch.setenv("LZF_GPU_KERNEL", "lane")
    monkeypatch.setenv("LZF_GPU_DECOMPRESS", "lane")
    streams = [b"", b"\x00", b"\xe0\x00\x00", b"\x1f" + b"q" * 31, b"\x00z\xa0\x00"]
    for cap in (0, 1, 7, 8, 32, 4096):
        dec = gpu_decompress(streams, [cap] * len(streams), align=3)
        for s_, d in zip(streams, dec):
            assert d == oracle.decompress(s_, cap), (s_, cap)
    rnd = random.Random(9)
    vals = [synth(rnd.randrange(6), 0x5EED00E0, i, rnd.randint(1, 9000)) for i in range(500)]
    streams = [oracle.compress(v, len(v) + len(v) // 16 + 64) for v in vals]
    assert all(streams)
    assert gpu_decompress(streams, [len(v) for v in vals], align=1) == [(v, 0) for v in vals]


@pytest.mark.parametrize("align", [1, 3])
def test_unaligned_arenas(oracle, generation, align):
    # values, streams and outputs at arbitrary byte offsets of their arenas
    from tests.gpu_batch import gpu_compress, gpu_decompress
    rnd = random.Random(align)
    vals, caps = [], []
    for i in range(600):
        n = rnd.choice([1, 2, 3, 4, 5, 17, 33, 64, 700, 4095, 4096])   # one size class
        vals.append(synth(rnd.randrange(6), 0x5EED00C0, i, n))
        caps.append(rnd.choice([max(1, n - 4), n + n // 16 + 64, rnd.randint(1, n + 8)]))
    res = gpu_compress(vals, caps, align=align)
    exp = [oracle.compress(v, c) for v, c in zip(vals, caps)]
    bad = [i for i, (a, b) in enumerate(zip(res, exp)) if a != b]
    assert not bad, f"{len(bad)} mismatches; first {bad[:5]}"
    streams = [r for r in exp if r]
    origs = [v for v, r in zip(vals, exp) if r]
    assert gpu_decompress(streams, [len(v) for v in origs], align=align) == [(v, 0) for v in origs]


def test_lane_mid_class(oracle, monkeypatch, diag):
    # the mid-class lane kernels (values 4 KiB .. 64 KiB), opt-in
    from tests.gpu_batch import gpu_compress
    monkeypatch.setenv("LZF_GPU_KERNEL", "lane")
    monkeypatch.setenv("LZF_GPU_CAND", "small")
    monkeypatch.setenv("LZF_GPU_LANE_MID", "1")
    monkeypatch.setenv("LZF_GPU_LANE_RING", "0")
    rnd = random.Random(21)
    vals = [synth(rnd.randrange(6), 0x5EED00F0, i, rnd.randint(1, 20000)) for i in range(300)]
    caps = [rnd.choice([max(1, len(v) - 4), len(v) + len(v) // 16 + 64]) for v in vals]
    assert gpu_compress(vals, caps, align=3) == [oracle.compress(v, c) for v, c in zip(vals, caps)]


@pytest.mark.parametrize("align", [16, 3])
def test_lane_ring_class(oracle, monkeypatch, align, diag):
    # the ring form of the cand kernel (values 8-64 KiB): links kept for the
    # last 8 KiB of positions, window tests on heads and links, and past
    # 16 KiB the bytes streamed through an LDS ring
    from tests.gpu_batch import gpu_compress, gpu_decompress
    monkeypatch.setenv("LZF_GPU_KERNEL", "lane")
    monkeypatch.setenv("LZF_GPU_CAND", "small")
    monkeypatch.setenv("LZF_GPU_LANE_RING", "1")
    rnd = random.Random(33 + align)
    vals = []
    for i in range(1500):
        n = rnd.choice([rnd.randint(1, 700), rnd.randint(8000, 16384), 16384,
                         rnd.randint(16385, 65536), 65536])
        v = synth(rnd.randrange(6), 0x5EED00F8, i, n)
        if rnd.random() < 0.1:
            v = bytes(rnd.choice(b"abc") for _ in range(n))
        vals.append(v)
    caps = [rnd.choice([max(1, len(v) - 4), len(v) + len(v) // 16 + 64, rnd.randint(1, len(v) + 64)])
            for v in vals]
    exp = [oracle.compress(v, c) for v, c in zip(vals, caps)]
    assert gpu_compress(vals, caps, align=align) == exp
    streams = [r for r in exp if r]
    origs = [v for v, r in zip(vals, exp) if r]
    assert gpu_decompress(streams, [len(v) for v in origs]) == [(v, 0) for v in origs]


def _chunks():
    # scratch chunks of this thread's last scratch-bound compress launch
    import re
    import gibson_amd
    m = re.search(r"scratch_chunks=(\d+)", gibson_amd.kernel_info())
    return int(m.group(1)) if m else 0


def _chunked_compress(oracle, vals, caps):
    # the scratch is one per device, shared by every thread, and earlier tests
    # grew it far past 1 MiB: the cap must still bind (the buffer is re-made
    # at it), and the launch must really have run in several chunks
    from tests.gpu_batch import gpu_compress
    assert gpu_compress(vals, caps, align=3) == [oracle.compress(v, c) for v, c in zip(vals, caps)]
    n = _chunks()
    assert n > 1, f"scratch_chunks={n}"
    return n


@pytest.mark.parametrize("nmax", [4096, 8192, 16384, 65536])
@pytest.mark.parametrize("cand", ["stream", "small"])
def test_lane_scratch_chunks(oracle, monkeypatch, nmax, cand, diag):
    # a 1 MiB compress scratch cap runs the lane kernels over many chunks
    monkeypatch.setenv("LZF_GPU_KERNEL", "lane")
    monkeypatch.setenv("LZF_GPU_CAND", cand)
    monkeypatch.setenv("LZF_GPU_SCRATCH_MB", "1")
    rnd = random.Random(nmax)
    vals = [synth(rnd.randrange(6), 0x5EED00FA, i, rnd.randint(1, nmax)) for i in range(400)]
    _chunked_compress(oracle, vals, [max(1, len(v) - 4) for v in vals])


@pytest.mark.parametrize("nmax", [4096, 65536])
@pytest.mark.parametrize("gen", ["table", "wtab"])
def test_table_scratch_chunks(oracle, monkeypatch, nmax, gen):
    # the table generation (and the window generation, diagnostic build)
    # over many scratch chunks
    monkeypatch.setenv("LZF_GPU_KERNEL", gen)
    monkeypatch.setenv("LZF_GPU_SCRATCH_MB", "1")
    rnd = random.Random(nmax + 1)
    vals = [synth(rnd.randrange(6), 0x5EED00FB, i, rnd.randint(1, nmax)) for i in range(300)]
    caps = [max(1, len(v) - 4) for v in vals]
    if gen == "wtab":
        with _diag():
            _chunked_compress(oracle, vals, caps)
    else:
        _chunked_compress(oracle, vals, caps)


def test_scratch_chunks_default_route(oracle, monkeypatch):
    # the product routing (lane generation, stream cand kernel) under a cap
    monkeypatch.delenv("LZF_GPU_KERNEL", raising=False)
    monkeypatch.setenv("LZF_GPU_SCRATCH_MB", "1")
    rnd = random.Random(99)
    vals = [synth(rnd.randrange(6), 0x5EED00FC, i, rnd.randint(1, 16384)) for i in range(300)]
    _chunked_compress(oracle, vals, [max(1, len(v) - 4) for v in vals])


@pytest.mark.parametrize("n", [8192, 16384])
def test_default_route_with_small_cand_knob(oracle, monkeypatch, diag, n):
    # LZF_GPU_CAND=small (diagnostic) takes values of at most 4 KiB: the
    # default routing then sends 8 / 16 KiB batches to the table generation
    # instead of failing the launch
    monkeypatch.delenv("LZF_GPU_KERNEL", raising=False)
    monkeypatch.setenv("LZF_GPU_CAND", "small")
    monkeypatch.setenv("LZF_GPU_LANE_RING", "0")
    rnd = random.Random(n)
    vals = [synth(rnd.randrange(6), 0x5EED00FD, i, rnd.randint(n // 2, n)) for i in range(200)]
    caps = [max(1, len(v) - 4) for v in vals]
    from tests.gpu_batch import gpu_compress
    assert gpu_compress(vals, caps) == [oracle.compress(v, c) for v, c in zip(vals, caps)]


@pytest.mark.parametrize("align", [16, 3])
def test_wave_parse(oracle, monkeypatch, align, diag):
    # the wave form of the parse kernel (64 positions per step, opt-in):
    # every size class edge of a window, caps that run out inside a window
    from tests.gpu_batch import gpu_compress
    monkeypatch.setenv("LZF_GPU_KERNEL", "lane")
    monkeypatch.setenv("LZF_GPU_CAND", "small")
    monkeypatch.setenv("LZF_GPU_LANE_PARSE", "wave")
    rnd = random.Random(77 + align)
    vals = [synth(rnd.randrange(6), 0x5EED00E0, i, rnd.randint(1, 4096)) for i in range(400)]
    vals += [synth(k, 0x5EED00E1, n, n) for k in range(6) for n in (1, 2, 3, 4, 5, 63, 64, 65, 66, 67, 130)]
    caps = [rnd.choice([max(1, len(v) - 4), len(v) + len(v) // 16 + 64, rnd.randint(1, len(v) + 8)]) for v in vals]
    assert gpu_compress(vals, caps, align=align) == [oracle.compress(v, c) for v, c in zip(vals, caps)]


def test_small_batch_routing(oracle, monkeypatch):
    # default threshold: a small batch compresses with the window generation,
    # bit-exact like the rest
    from tests.gpu_batch import gpu_compress
    monkeypatch.delenv("LZF_GPU_KERNEL", raising=False)
    monkeypatch.delenv("LZF_GPU_LANE_MIN", raising=False)
    rnd = random.Random(5)
    vals = [synth(rnd.randrange(6), 0x5EED00C0, i, rnd.randint(1, 4096)) for i in range(200)]
    caps = [max(1, len(v) - 4) for v in vals]
    assert gpu_compress(vals, caps) == [oracle.compress(v, c) for v, c in zip(vals, caps)]


def test_lane_order_repair_path(oracle, monkeypatch, diag):
    # the repair path of the bucket-head atomics (taken when the LDS does not
    # serialise a wave's same-address atomics in lane order) gives the same
    # streams
    from tests.gpu_batch import gpu_compress
    monkeypatch.setenv("LZF_GPU_KERNEL", "lane")
    monkeypatch.setenv("LZF_GPU_CAND", "small")
    monkeypatch.setenv("LZF_GPU_LANE_FORCE_FIX", "1")
    monkeypatch.setenv("LZF_GPU_LANE_MID", "1")
    monkeypatch.setenv("LZF_GPU_LANE_RING", "0")
    rnd = random.Random(3)
    for nmax in (4096, 20000):
        vals = [synth(rnd.randrange(6), 0x5EED00D0, i, rnd.randint(1, nmax)) for i in range(200)]
        caps = [max(1, len(v) - 4) for v in vals]
        assert gpu_compress(vals, caps) == [oracle.compress(v, c) for v, c in zip(vals, caps)]


@pytest.mark.parametrize("nmax", [4096, 8192, 9000, 16384, 65536])
def test_random_differential(oracle, generation, nmax, monkeypatch):
    # nmax 8192: the batch fits the non-wrapping ring/chain kernel; 9000:
    # the wrapping one (the kernel is chosen per batch from max_len); 16384
    # takes the lane generation's ring class
    from tests.gpu_batch import gpu_compress, gpu_decompress
    if nmax >= 16384:
        monkeypatch.setenv("LZF_GPU_LANE_RING", "1")
    rnd = random.Random(7 + nmax)
    vals, caps = [], []
    for it in range(3000):
        kind = rnd.randrange(6)
        n = rnd.choice([rnd.randint(1, 64), rnd.randint(1, 700), rnd.randint(1, nmax)])
        v = synth(kind, rnd.getrandbits(32), it, n)
        if rnd.random() < 0.2:
            v = bytes(rnd.choice(b"ab") for _ in range(n))
        vals.append(v)
        caps.append(rnd.choice([max(1, n - 4), n + n // 16 + 64, rnd.randint(1, n + 64)]))
    res = gpu_compress(vals, caps)
    exp = [oracle.compress(v, c) for v, c in zip(vals, caps)]
    bad = [i for i, (a, b) in enumerate(zip(res, exp)) if a != b]
    assert not bad, f"{len(bad)} mismatches; first {bad[:5]}"
    streams = [r for r in exp if r]
    origs = [v for v, r in zip(vals, exp) if r]
    dec = gpu_decompress(streams, [len(v) for v in origs])
    assert all(d == (v, 0) for d, v in zip(dec, origs))


def test_edge_cases(oracle):
    from tests.gpu_batch import gpu_compress, gpu_decompress
    vals = [b"", b"x", b"x", b"ab", b"abc", b"a" * 5, b"a" * 300, b"\0" * 65536,
            bytes(range(256)) * 4, b"ab" * 4000]
    caps = [10, 3, 4, 5, 6, 1, 296, 65532, 1020, 8000]
    res = gpu_compress(vals, caps)
    for v, c, r in zip(vals, caps, res):
        assert r == oracle.compress(v, c), (len(v), c)
    streams = [b"", b"\x00", b"\xe0\x00\x00", b"\x1f" + b"q" * 31, b"\x00z\xa0\x00"]
    for cap in (0, 1, 7, 8, 32, 4096):
        dec = gpu_decompress(streams, [cap] * len(streams))
        for s, d in zip(streams, dec):
            # phantom control byte 0xff for the empty stream, as in tests/golden
            o, e = oracle.decompress(s, cap)
            assert d == (o, e), (s, cap, d, (o, e))


def test_large_values(oracle, generation):
    # values past the 16 KiB ring (wrapping ring and chain) and past 64 KiB
    # (64-bit bucket heads), up to 1 MiB
    from tests.gpu_batch import gpu_compress, gpu_decompress
    if generation == "serial":
        pytest.skip("the serial kernel is limited to 64 KiB")
    rnd = random.Random(11)
    vals, caps = [], []
    for k, n in enumerate([16385, 70000, 65537, 200003, 1 << 20]):
        v = synth(k % 6, 0x5EED00AA, k, n)
        if k == 3:
            v = bytes(rnd.choice(b"abc") for _ in range(n))
        vals.append(v)
        caps.append(n - 4)
    res = gpu_compress(vals, caps)
    for v, c, r in zip(vals, caps, res):
        assert r == oracle.compress(v, c), len(v)
    streams = [r for r in res if r]
    origs = [v for v, r in zip(vals, res) if r]
    assert streams
    assert gpu_decompress(streams, [len(v) for v in origs]) == [(v, 0) for v in origs]


def test_device_generator_matches_host():
    import gibson_amd
    for kind in range(6):
        for n in (1, 37, 4096, 16384):
            out = torch.zeros(3 * n, dtype=torch.uint8, device="cuda")
            gibson_amd.synth_fill(kind, 0x5EED0002, 5, 7, 3, n, out)
            torch.cuda.synchronize()
            host = b"".join(synth(kind, 0x5EED0002, 5 + 7 * k, n) for k in range(3))
            assert bytes(out.cpu().numpy()) == host, (kind, n)


# ---- BASELINE.json sizes: bit-exact over whole batches ----------------------

CONFIGS = [
    # (kind, seed, n, count): the first 64 K values of configs[1..4], and all
    # 256 K values of configs[2] (one scratch chunk); every stream of every
    # value is checked against the reference's digest (tests/golden/digests.json)
    (1, 0x5EED0002, 4096, 65536),
    (2, 0x5EED0003, 65536, 65536),
    (2, 0x5EED0003, 65536, 262144),  # the table generation (values past 16 KiB)
    (0, 0x5EED0004, 8192, 65536),
    (3, 0x5EED0005, 16384, 65536),
    # the production routes at the configs' real per-GPU counts: 262 144
    # values of 4 KiB and 131 072 of 16 KiB run the lane generation with the
    # stream cand kernel (below 163 840 / 81 920 values both would run window64)
    (1, 0x5EED0002, 4096, 262144),
    (3, 0x5EED0005, 16384, 131072),
]


@pytest.fixture(scope="module")
def digests():
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "digests.json")) as f:
        return {(d["kind"], d["seed"], d["n"], d["count"]): d["sha256"] for d in json.load(f)["digests"]
                if not d.get("first")}


@pytest.mark.parametrize("kind,seed,n,count", CONFIGS)
def test_full_batch_digest_and_roundtrip(kind, seed, n, count, digests, monkeypatch):
    monkeypatch.delenv("LZF_GPU_LANE_MIN", raising=False)      # the routing the bench uses
    _digest_case(kind, seed, n, count, digests)


@pytest.mark.parametrize("kind,seed,n,count", [c for c in CONFIGS if c[2] <= 16384 and c[3] >= 131072])
@pytest.mark.parametrize("gen", ["table", "lane-small"])
def test_full_batch_digest_other_cand(kind, seed, n, count, gen, digests, monkeypatch):
    # the production-size digests through the generations the routing no
    # longer takes there: the table generation, and (4 KiB, diagnostic build)
    # the small class
    if gen == "lane-small" and n > 4096:
        pytest.skip("the small class takes values of at most 4 KiB")
    monkeypatch.delenv("LZF_GPU_LANE_MIN", raising=False)
    for k, v in GEN_ENV[gen].items():
        monkeypatch.setenv(k, v)
    if gen in DIAG:
        with _diag():
            _digest_case(kind, seed, n, count, digests)
    else:
        _digest_case(kind, seed, n, count, digests)


@pytest.mark.parametrize("kind,seed,n,count", [c for c in CONFIGS if c[3] <= 65536])
def test_full_batch_digest_wtab(kind, seed, n, count, digests, monkeypatch, diag):
    monkeypatch.setenv("LZF_GPU_KERNEL", "wtab")
    _digest_case(kind, seed, n, count, digests)


# the configs' real counts (round 5): all 1 048 576 values of configs[1], the
# first 1 M-value chunk of configs[4] (the chunk bench.py runs), and 1 M
# values of configs[3] whose decoded output is also checked against the
# reference decoder's (decoded_sha256)
FULL = [(1, 0x5EED0002, 4096, 1048576), (3, 0x5EED0005, 16384, 1048576), (0, 0x5EED0004, 8192, 1048576)]


@pytest.mark.parametrize("kind,seed,n,count", FULL)
def test_full_count_digest(kind, seed, n, count, digests, monkeypatch):
    import json
    monkeypatch.delenv("LZF_GPU_LANE_MIN", raising=False)
    with open(os.path.join(os.path.dirname(__file__), "golden", "digests.json")) as f:
        rec = {(d["kind"], d["seed"], d["n"], d["count"]): d for d in json.load(f)["digests"] if not d.get("first")}
    _digest_case(kind, seed, n, count, digests, decoded=rec[(kind, seed, n, count)].get("decoded_sha256"))


# round 6: the rest of the configs' real counts, one 1 M-value chunk per test
# -- configs[3]'s values 1 M .. 8 M (streams and the reference decoder's
# output), configs[4]'s values 1 M .. 4 M -- so every value of configs[1],
# [3] and [4] and all of configs[2] is checked against the reference
CHUNKS = [(0, 0x5EED0004, 8192, k << 20) for k in range(1, 8)] + [(3, 0x5EED0005, 16384, k << 20) for k in range(1, 4)]


@pytest.mark.parametrize("kind,seed,n,first", CHUNKS, ids=[f"k{c[0]}-{c[2]}-{c[3] >> 20}M" for c in CHUNKS])
def test_full_count_digest_chunk(kind, seed, n, first, monkeypatch):
    import json
    monkeypatch.delenv("LZF_GPU_LANE_MIN", raising=False)
    count = 1 << 20
    with open(os.path.join(os.path.dirname(__file__), "golden", "digests.json")) as f:
        rec = {(d["kind"], d["seed"], d["n"], d.get("first", 0), d["count"]): d for d in json.load(f)["digests"]}
    r = rec[(kind, seed, n, first, count)]
    _digest_case(kind, seed, n, count, {(kind, seed, n, count): r["sha256"]}, decoded=r.get("decoded_sha256"),
                 first=first)


@pytest.mark.parametrize("gen,chunks", [("default", 3), ("table", 5)])
def test_full_batch_digest_chunked_scratch(digests, monkeypatch, gen, chunks):
    # configs[2]'s 262 144 x 64 KiB under a 16 GiB scratch cap (a GPU-sharing
    # server's route), bit-exact by the reference's digest: by default the
    # lane generation, whose half-size scratch needs three chunks where the
    # table generation (forced) needs five
    monkeypatch.delenv("LZF_GPU_LANE_MIN", raising=False)
    monkeypatch.setenv("LZF_GPU_SCRATCH_MB", "16384")
    if gen == "table":
        monkeypatch.setenv("LZF_GPU_KERNEL", "table")
    _digest_case(2, 0x5EED0003, 65536, 262144, digests)
    assert _chunks() == chunks, _chunks()


def _digest_case(kind, seed, n, count, digests, decoded=None, first=0):
    import gibson_amd
    from tests.digest import batch_digest
    dev = "cuda"
    src = torch.empty(count * n, dtype=torch.uint8, device=dev)
    gibson_amd.synth_fill(kind, seed, first, 1, count, n, src)
    in_off = torch.arange(count, dtype=torch.int64, device=dev) * n
    in_len = torch.full((count,), n, dtype=torch.int32, device=dev)
    cap = torch.full((count,), n - 4, dtype=torch.int32, device=dev)
    comp = torch.zeros(count * n, dtype=torch.uint8, device=dev)
    clen = torch.zeros(count, dtype=torch.int32, device=dev)
    gibson_amd.compress_batch(src, in_off, in_len, comp, in_off, cap, clen, n)
    torch.cuda.synchronize()
    # every value's stream, bit-exact with the reference (whole-batch digest)
    assert batch_digest(comp.cpu().numpy(), n, clen.cpu().numpy()) == digests[(kind, seed, n, count)]
    # round trip identity on every compressed value
    dec = torch.zeros(count * n, dtype=torch.uint8, device=dev)
    dlen = torch.zeros(count, dtype=torch.int32, device=dev)
    err = torch.zeros(count, dtype=torch.int32, device=dev)
    ok = clen > 0
    dcap = torch.where(ok, torch.full_like(clen, n), torch.zeros_like(clen))
    gibson_amd.decompress_batch(comp, in_off, torch.where(ok, clen, torch.ones_like(clen)),
                                dec, in_off, dcap, dlen, err, n)
    torch.cuda.synchronize()
    if decoded is not None:
        # the decoder's output, every value, against the reference decoder's
        del comp
        dl = torch.where(ok, dlen, torch.zeros_like(dlen)).cpu().numpy()
        assert batch_digest(dec.cpu().numpy(), n, dl) == decoded
    assert torch.equal(dlen[ok], torch.full_like(dlen[ok], n))
    for r0 in range(0, count, 16384):
        r1 = min(count, r0 + 16384)
        d, sv, o = dec.view(count, n)[r0:r1], src.view(count, n)[r0:r1], ok[r0:r1]
        assert not bool(((d != sv).any(dim=1) & o).any())
    assert int(ok.sum()) > 0


def test_host_batch_pipelined(oracle):
    # a host batch of 96 MiB runs the chunked two-slot pipeline: values in
    # shuffled, unaligned arena order with mixed sizes, checked against the
    # oracle (a sample) and by the round trip (all)
    import gibson_amd
    rnd = random.Random(17)
    count = 24000
    sizes = [rnd.choice([4096, 4096, 4096, rnd.randint(1, 8192)]) for _ in range(count)]
    order = list(range(count))
    rnd.shuffle(order)
    pos, offs = 0, [0] * count
    for i in order:
        offs[i] = pos
        pos += sizes[i] + rnd.randint(0, 3)
    arena = np.zeros(pos + 16, np.uint8)
    kinds = [rnd.randrange(6) for _ in range(count)]
    for i in range(count):
        arena[offs[i]:offs[i] + sizes[i]] = np.frombuffer(synth(kinds[i], 0x5EED00B0, i, sizes[i]), np.uint8)
    off = np.array(offs, dtype=np.uint64)
    ln = np.array(sizes, dtype=np.uint32)
    cap = np.maximum(ln.astype(np.int64) - 4, 1).astype(np.uint32)
    out = np.zeros_like(arena)
    olen = np.zeros(count, np.uint32)
    gibson_amd.host_compress_batch(arena, off, ln, out, off, cap, olen)
    for i in rnd.sample(range(count), 400):
        v = bytes(arena[offs[i]:offs[i] + sizes[i]])
        exp = oracle.compress(v, int(cap[i]))
        got = bytes(out[offs[i]:offs[i] + olen[i]]) if olen[i] else None
        assert got == exp, i
    ok = olen > 0
    dec = np.zeros_like(arena)
    dl = np.zeros(int(ok.sum()), np.uint32)
    er = np.zeros(int(ok.sum()), np.int32)
    gibson_amd.host_decompress_batch(out, off[ok], olen[ok], dec, off[ok], ln[ok], dl, er)
    assert (dl == ln[ok]).all() and (er == 0).all()
    for i in np.nonzero(ok)[0][:2000]:
        assert bytes(dec[offs[i]:offs[i] + sizes[i]]) == bytes(arena[offs[i]:offs[i] + sizes[i]])


def test_host_batch_api(oracle):
    import gibson_amd
    vals = [synth(1, 11, i, 4096) for i in range(64)] + [synth(4, 11, 0, 4096)]
    arena = np.frombuffer(b"".join(vals), np.uint8).copy()
    off = np.arange(len(vals), dtype=np.uint64) * 4096
    ln = np.full(len(vals), 4096, np.uint32)
    cap = np.full(len(vals), 4092, np.uint32)
    out = np.zeros_like(arena)
    olen = np.zeros(len(vals), np.uint32)
    gibson_amd.host_compress_batch(arena, off, ln, out, off, cap, olen)
    for i, v in enumerate(vals):
        exp = oracle.compress(v, 4092)
        got = bytes(out[off[i]:off[i] + olen[i]]) if olen[i] else None
        assert got == exp
    dec = np.zeros_like(arena)
    dl = np.zeros(len(vals), np.uint32)
    er = np.zeros(len(vals), np.int32)
    ok = olen > 0
    gibson_amd.host_decompress_batch(out, off[ok], olen[ok], dec, off[ok], ln[ok], dl, er)
    assert (dl[:ok.sum()] == 4096).all() and (er[:ok.sum()] == 0).all()


def test_decode_self_overlapping_references(oracle):
    # runs of every period 1..70 (a back-reference whose distance is below its
    # length repeats its last d bytes, src/lzf_d.c:137-142), starting at
    # every phase of a 64-byte output group, inside values past 4 KiB so the
    # two-wave decoder (and its periodic-source path, CD_PERIOD) decodes them
    from tests.gpu_batch import gpu_decompress
    rnd = random.Random(70)
    vals = []
    for period in range(1, 71):
        for phase in (0, 1, 17, 63):
            pat = bytes(rnd.randrange(256) for _ in range(period))
            head = bytes(rnd.randrange(256) for _ in range(4096 + phase))
            body = (pat * (20000 // period + 2))[:rnd.randint(300, 12000)]
            tail = synth(0, 0x5EED0DD0, period * 4 + phase, rnd.randint(100, 3000))
            vals.append(head + body + tail)
    streams = [oracle.compress(v, len(v) + len(v) // 16 + 64) for v in vals]
    assert all(streams)
    assert gpu_decompress(streams, [len(v) for v in vals]) == [(v, 0) for v in vals]


@pytest.mark.parametrize("nmax,align", [(8192, 16), (16384, 16), (16385, 16), (16384, 3)])
def test_decode_far_sources(oracle, nmax, align):
    # batches whose largest value is 4-16 KiB decode on the 4 KiB tokpar
    # window with sources more than 4 KiB behind the output group read back
    # from dst in HBM (CD_FAR_MAX); 16385 takes the 8 KiB pipe instead.  A
    # random block repeated at distances 4095..8192 (the LZF maximum, src/
    # lzf_d.c:121) puts copies on both sides of the window edge, self-
    # overlapping runs straddle it, and values at the batch maximum share the
    # launch with tiny ones; align 3 packs streams and output regions at
    # multiples of 3 bytes (far loads and 16-byte flushes off alignment)
    from tests.gpu_batch import gpu_decompress
    rnd = random.Random(nmax)
    vals = []
    for dist in (4095, 4096, 4097, 4100, 4160, 5000, 6144, 8000, 8191, 8192):
        for phase in (0, 5, 63):
            blk = bytes(rnd.randrange(256) for _ in range(dist))
            v = bytes(rnd.randrange(256) for _ in range(phase)) + blk
            while len(v) < nmax:
                v += blk[:rnd.randint(3, 300)] + bytes(rnd.randrange(256) for _ in range(rnd.randint(0, 40)))
            vals.append(v[:nmax - rnd.randrange(0, 64)])
    for period in (1, 2, 7, 64, 65):
        head = bytes(rnd.randrange(256) for _ in range(4090))
        pat = bytes(rnd.randrange(256) for _ in range(period))
        vals.append((head + pat * (nmax // period + 1))[:nmax])
    vals += [b"", b"a", synth(0, 0xFA2, 1, 300), synth(1, 0xFA2, 2, nmax)]
    vals.append(vals[0][:nmax])
    streams = [oracle.compress(v, len(v) + len(v) // 16 + 64) if v else b"" for v in vals]
    assert all(s or not v for s, v in zip(streams, vals))
    keep = [i for i, v in enumerate(vals) if v]
    got = gpu_decompress([streams[i] for i in keep], [len(vals[i]) for i in keep], align=align)
    assert got == [(vals[i], 0) for i in keep]
    # the same streams truncated: the errno the reference returns on the
    # FAR route's batches (src/lzf_d.c:79-82, 110-114, 127-130)
    bad_s, bad_l = [], []
    for i in keep[:12]:
        s = streams[i]
        bad_s.append(s[:len(s) * 2 // 3])
        bad_l.append(len(vals[i]))
    res = gpu_decompress(bad_s, bad_l, align=align)
    for s, n, (out, e) in zip(bad_s, bad_l, res):
        ref = oracle.decompress(s, n)
        assert (out, e) == ref
