"""ctypes mirror of include/gb_batch.h: Gibson's SET/MSET/MGET codec call
sites as device batches (src/query.c:374-425, :479-502; src/net.c:1256-1342),
plus the original-length side table."""
import ctypes

import numpy as np

from .lzf import _ERRS, lib

ENC_PLAIN, ENC_LZF, ENC_NUMBER, ENC_NULL = 0x00, 0x01, 0x02, 0xFF


class Stats(ctypes.Structure):
    _fields_ = [("compravg", ctypes.c_double), ("ncompressed", ctypes.c_uint64)]


class Stored(ctypes.Structure):
    _fields_ = [("encoding", ctypes.c_uint8), ("size", ctypes.c_uint32), ("orig_len", ctypes.c_uint32)]


_BOUND = set()


def _L():
    L = lib()
    if id(L) in _BOUND:
        return L
    vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
    L.gb_set_batch.restype = ctypes.c_int
    L.gb_set_batch.argtypes = [vp, vp, vp, u32, u32, vp, vp, vp, vp]
    L.gb_mset.restype = ctypes.c_int
    L.gb_mset.argtypes = [vp, u32, u32, u32, vp, vp, vp]
    L.gb_mget_payload.restype = ctypes.c_long
    L.gb_mget_payload.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, u32, u32, u32, u64, ctypes.c_int, vp]
    L.gb_lentab_new.restype = vp
    L.gb_lentab_new.argtypes = []
    L.gb_lentab_free.restype = None
    L.gb_lentab_free.argtypes = [vp]
    L.gb_lentab_put.restype = ctypes.c_int
    L.gb_lentab_put.argtypes = [vp, u64, u32]
    L.gb_lentab_get.restype = ctypes.c_int
    L.gb_lentab_get.argtypes = [vp, u64, ctypes.POINTER(u32)]
    L.gb_lentab_del.restype = ctypes.c_int
    L.gb_lentab_del.argtypes = [vp, u64]
    L.gb_lentab_size.restype = ctypes.c_size_t
    L.gb_lentab_size.argtypes = [vp]
    L.gb_mget_last_staged.restype = u64
    L.gb_mget_last_staged.argtypes = []
    _BOUND.add(id(L))
    return L


def _check(rc, what):
    if rc < 0:
        raise RuntimeError(f"{what} failed: {_ERRS.get(rc, rc)}")


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def set_batch(values, compression, stats=None):
    """gbSingleSet's store decision for each value: [(encoding, stored bytes,
    orig_len)], one device batch for the values above ``compression``."""
    n = len(values)
    arena = np.frombuffer(b"".join(values) + b"\0" * 8, np.uint8).copy()
    v_len = np.array([len(v) for v in values], np.uint32)
    v_off = np.concatenate([[0], np.cumsum(v_len[:-1])]).astype(np.uint64)
    room = np.maximum(v_len.astype(np.int64) - 4, 8) + 16
    out_off = np.concatenate([[0], np.cumsum(room[:-1])]).astype(np.uint64)
    out = np.zeros(int(room.sum()) + 16, np.uint8)
    st = (Stored * n)()
    rc = _L().gb_set_batch(_p(arena), _p(v_off), _p(v_len), n, compression, _p(out), _p(out_off),
                           ctypes.cast(st, ctypes.c_void_p),
                           ctypes.cast(ctypes.pointer(stats), ctypes.c_void_p) if stats is not None else None)
    _check(rc, "gb_set_batch")
    res = []
    for i, v in enumerate(values):
        if st[i].encoding == ENC_LZF:
            o = int(out_off[i])
            res.append((ENC_LZF, bytes(out[o:o + st[i].size]), st[i].orig_len))
        else:
            res.append((ENC_PLAIN, v, st[i].orig_len))
    return res


def mset(value, nkeys, compression, stats=None):
    out = np.zeros(max(len(value) - 4, 8) + 16, np.uint8)
    src = np.frombuffer(value + b"\0" * 8, np.uint8).copy()
    st = Stored()
    rc = _L().gb_mset(_p(src), len(value), nkeys, compression, _p(out), ctypes.cast(ctypes.pointer(st), ctypes.c_void_p),
                      ctypes.cast(ctypes.pointer(stats), ctypes.c_void_p) if stats is not None else None)
    _check(rc, "gb_mset")
    if st.encoding == ENC_LZF:
        return ENC_LZF, bytes(out[:st.size]), st.orig_len
    return ENC_PLAIN, value, st.orig_len


def mget_payload(items, elements, maxrequestsize, max_response, orig_lens=None, reply_header=True):
    """items: [(key, enc, stored bytes)]; the MGET reply frame or None
    (CHECK_SPACE, or an LZF item that does not decode)."""
    n = len(items)
    keys = np.frombuffer(b"".join(k for k, _, _ in items) + b"\0", np.uint8).copy()
    vals = np.frombuffer(b"".join(v for _, _, v in items) + b"\0", np.uint8).copy()
    kl = np.array([len(k) for k, _, _ in items], np.uint32)
    vs = np.array([len(v) for _, _, v in items], np.uint32)
    ko = np.concatenate([[0], np.cumsum(kl[:-1])]).astype(np.uint64) if n else np.zeros(0, np.uint64)
    vo = np.concatenate([[0], np.cumsum(vs[:-1])]).astype(np.uint64) if n else np.zeros(0, np.uint64)
    en = np.array([e for _, e, _ in items], np.uint8)
    ol = np.array(orig_lens, np.uint32) if orig_lens is not None else None
    out = np.zeros(max_response + 16, np.uint8)
    r = _L().gb_mget_payload(_p(keys), _p(ko), _p(kl), _p(vals), _p(vo), _p(vs), _p(en),
                             _p(ol) if ol is not None else None, n, elements, maxrequestsize, max_response,
                             1 if reply_header else 0, _p(out))
    _check(r, "gb_mget_payload")
    return bytes(out[:r]) if r > 0 else None


def mget_last_staged():
    """Bytes of decode arena the last mget_payload of this thread staged."""
    return int(_L().gb_mget_last_staged())


class LenTab:
    """The original-length side table (gb_lentab_*)."""

    def __init__(self):
        self._L = _L()
        self._t = self._L.gb_lentab_new()
        if not self._t:
            raise MemoryError

    def __del__(self):
        if getattr(self, "_t", None):
            self._L.gb_lentab_free(self._t)
            self._t = None

    def put(self, item, orig_len):
        _check(self._L.gb_lentab_put(self._t, item, orig_len), "gb_lentab_put")

    def get(self, item):
        v = ctypes.c_uint32()
        return v.value if self._L.gb_lentab_get(self._t, item, ctypes.byref(v)) else None

    def delete(self, item):
        return bool(self._L.gb_lentab_del(self._t, item))

    def __len__(self):
        return int(self._L.gb_lentab_size(self._t))
