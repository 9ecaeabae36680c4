"""Gibson's SET/MSET/MGET call sites as device batches (include/gb_batch.h),
against the reference's per-key semantics restated from src/query.c:374-425,
:479-502 and src/net.c:1256-1342 (the codec bytes against the oracle, the
MGET payload against the oracle's frame restatement)."""
import random

import pytest

from tests.oracle_lib import synth

torch = pytest.importorskip("torch")


def _single_set(oracle, v, compression, stats):
    """gbSingleSet (src/query.c:374-425), one key."""
    if len(v) > compression:
        cap = (len(v) - 4) & 0xFFFFFFFF             # size_t vlen - 4 as unsigned int
        s = oracle.compress(v, min(cap, len(v) + len(v) // 16 + 8))
        if s:
            rate = 100.0 - ((len(s) * 100.0) / len(v))
            stats[0] = rate if stats[0] == 0 else (stats[0] + rate) / 2.0
            stats[1] += 1
            return (1, s, len(v))
    return (0, v, len(v))


def test_lentab_put_get_delete_grow():
    # pure host code: no device call
    from gibson_amd.gb import LenTab
    t = LenTab()
    rnd = random.Random(4)
    ref = {}
    for it in range(20000):
        k = rnd.getrandbits(64) if rnd.random() < 0.7 else rnd.choice(list(ref) or [1])
        op = rnd.random()
        if op < 0.6:
            ln = rnd.getrandbits(32)
            t.put(k, ln)
            ref[k] = ln
        elif op < 0.8:
            assert t.delete(k) == (k in ref)
            ref.pop(k, None)
        else:
            assert t.get(k) == ref.get(k)
    assert len(t) == len(ref)
    for k, v in ref.items():
        assert t.get(k) == v


@pytest.mark.gpu
def test_set_batch_matches_per_key_semantics(oracle):
    from gibson_amd.gb import Stats, set_batch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rnd = random.Random(8)
    compression = 4096                          # debian/etc/gibson/gibson.conf: compression 4K
    vals = []
    for i in range(3000):
        n = rnd.choice([1, 3, 5, 100, 4095, 4096, 4097, rnd.randint(4097, 70000), 65536])
        vals.append(synth(rnd.randrange(6), 0x5EED0A00, i, n))
    st = Stats()
    got = set_batch(vals, compression, st)
    ref_stats = [0.0, 0]
    exp = [_single_set(oracle, v, compression, ref_stats) for v in vals]
    assert got == exp
    assert st.compravg == ref_stats[0] and st.ncompressed == ref_stats[1]
    # small thresholds: values shorter than 4 bytes get the reference's wrapped out_len
    st2 = Stats()
    tiny = [b"a", b"ab", b"abc", b"abcd", b"abcde", b"aaaaaaaaaaaaaaaa"]
    ref2 = [0.0, 0]
    assert set_batch(tiny, 0, st2) == [_single_set(oracle, v, 0, ref2) for v in tiny]
    assert (st2.compravg, st2.ncompressed) == tuple(ref2)


@pytest.mark.gpu
@pytest.mark.parametrize("nkeys", [1, 2, 7, 100])
def test_mset_compresses_once_for_all_keys(oracle, nkeys):
    from gibson_amd.gb import Stats, mset
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    v = synth(2, 0x5EED0003, 5, 20000)
    st = Stats()
    st.compravg = 37.5
    got = mset(v, nkeys, 4096, st)
    ref = [37.5, 0]
    for _ in range(nkeys):                     # gbMultiSetCallback: one gbSingleSet per key
        e = _single_set(oracle, v, 4096, ref)
    assert got == e
    assert st.compravg == ref[0] and st.ncompressed == ref[1]
    assert mset(synth(4, 1, 1, 5000), nkeys, 4096)[0] == 0        # incompressible: stored plain


@pytest.mark.gpu
@pytest.mark.parametrize("side_table", [False, True])
def test_mget_payload_matches_reference_frame(oracle, side_table):
    from gibson_amd.gb import mget_payload
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rnd = random.Random(11 + side_table)
    items, lens = [], []
    for i in range(400):
        key = b"key:%d:" % i + bytes(rnd.choice(b"abcxyz") for _ in range(rnd.randint(1, 30)))
        kind = rnd.choice(["lzf", "lzf", "plain", "number", "null"])
        if kind == "lzf":
            v = synth(rnd.randrange(4), 0x5EED0A10, i, rnd.choice([4097, 9000, 65536]))
            s = oracle.compress(v, len(v) - 4)
            if s:
                items.append((key, 1, s))
                lens.append(len(v) if side_table else 0)
                continue
            kind = "plain"
        if kind == "plain":
            items.append((key, 0, synth(1, 0x5EED0A11, i, rnd.randint(1, 3000))))
        elif kind == "number":
            items.append((key, 2, rnd.getrandbits(63).to_bytes(8, "little")))
        else:
            items.append((key, 0xFF, b"\0"))
        lens.append(0)
    for maxresp in (1 << 30, 100000):
        for hdr in (True, False):
            exp = oracle.kv_frame(items, len(items), maxresp, 4 << 20, reply_header=hdr)
            got = mget_payload(items, len(items), 4 << 20, maxresp, orig_lens=lens, reply_header=hdr)
            assert got == exp


@pytest.mark.gpu
def test_mget_unknown_lengths_staged_exact(oracle):
    # 1000 LZF items with no side-table entry: the device pre-pass sizes
    # them, so the decode arena is their decoded bytes, not 1000 x 4 MiB
    # (the reference decodes each at out_len = maxrequestsize, src/net.c:1309)
    from gibson_amd.gb import mget_last_staged, mget_payload
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rnd = random.Random(21)
    items, decoded = [], 0
    for i in range(1000):
        v = synth(rnd.randrange(4), 0x5EED0A20, i, rnd.choice([300, 4096, 20000]))
        s = oracle.compress(v, len(v) + len(v) // 16 + 64)
        assert s
        items.append((b"k%d" % i, 1, s))
        decoded += len(v)
    exp = oracle.kv_frame(items, len(items), 1 << 30, 4 << 20)
    got = mget_payload(items, len(items), 4 << 20, 1 << 30, orig_lens=[0] * len(items))
    assert got == exp
    staged = mget_last_staged()
    assert decoded <= staged < 2 * decoded, (staged, decoded)
    # a payload known to exceed max_response stages nothing
    assert mget_payload(items, len(items), 4 << 20, 100000) is None
    assert mget_last_staged() == 0


@pytest.mark.gpu
def test_mget_stale_and_oversize_side_table(oracle):
    # side-table lengths that are too small (stale) are re-sized by the
    # pre-pass; an item longer than maxrequestsize does not decode and goes
    # out with size 0, as the release build of src/net.c:1306-1335 does
    from gibson_amd.gb import mget_payload
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rnd = random.Random(22)
    items, lens = [], []
    for i in range(60):
        v = synth(rnd.randrange(4), 0x5EED0A21, i, rnd.choice([500, 3000, 9000]))
        s = oracle.compress(v, len(v) + len(v) // 16 + 64)
        items.append((b"key%d" % i, 1, s))
        lens.append(rnd.choice([len(v), max(1, len(v) // 2), len(v) + 7, 0]))
    for maxreq in (4 << 20, 4096):
        exp = oracle.kv_frame(items, len(items), 1 << 30, maxreq)
        got = mget_payload(items, len(items), maxreq, 1 << 30, orig_lens=lens)
        assert got == exp, maxreq
