"""Test-side access to the CPU oracle (oracle/liblzf_oracle.so), the compiled
reference (oracle/_ref/liblzf_ref.so, when present) and the host synthetic
generator.  Checker only -- never used by the product path."""
import ctypes
import hashlib
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liblzf_oracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "liblzf_ref.so")
SYNTH_SO = os.path.join(ROOT, "gibson_amd", "libgibson_synth.so")


def _ensure_built():
    if not os.path.exists(ORACLE_SO):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "liblzf_oracle.so"])
    if not os.path.exists(SYNTH_SO):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "gibson_amd", "csrc"),
                               "../libgibson_synth.so"])


_ensure_built()
_SYN = ctypes.CDLL(SYNTH_SO)
_SYN.synth_fill.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                            ctypes.c_uint32, ctypes.c_void_p]


def synth(kind, seed, index, n):
    buf = ctypes.create_string_buffer(max(n, 1))
    _SYN.synth_fill(kind, seed, index, 1, n, buf)
    return buf.raw[:n]


def sha16(b):
    return hashlib.sha256(b).hexdigest()[:16]


class _Codec:
    def __init__(self, path, cname, dname):
        L = ctypes.CDLL(path, use_errno=True)
        self.c = getattr(L, cname)
        self.d = getattr(L, dname)
        for f in (self.c, self.d):
            f.restype = ctypes.c_uint
            f.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p, ctypes.c_uint]

    def compress(self, data, out_len):
        src = ctypes.create_string_buffer(data + b"\0" * 8, len(data) + 8)
        dst = ctypes.create_string_buffer(out_len + 16)
        r = self.c(src, len(data), dst, out_len)
        return dst.raw[:r] if r else None

    def decompress(self, data, out_len):
        src = ctypes.create_string_buffer(data + b"\xff", len(data) + 1)
        dst = ctypes.create_string_buffer(out_len + 16)
        ctypes.set_errno(0)
        r = self.d(src, len(data), dst, out_len)
        return (dst.raw[:r], 0) if r else (None, ctypes.get_errno())


class Oracle(_Codec):
    def __init__(self):
        super().__init__(ORACLE_SO, "oracle_lzf_compress", "oracle_lzf_decompress")
        L = ctypes.CDLL(ORACLE_SO)
        vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
        self.f = L.oracle_kv_frame
        self.f.restype = ctypes.c_long
        self.f.argtypes = [vp, vp, vp, vp, vp, vp, vp, u32, u32, u64, u32, ctypes.c_int, vp]

    def kv_frame(self, items, elements, max_response, maxrequestsize, reply_header=True):
        """items: [(key bytes, enc, stored bytes)]; the MGET reply frame
        (src/net.c:1256-1342) or None where CHECK_SPACE fails."""
        import numpy as np
        keys = b"".join(k for k, _, _ in items) or b"\0"
        vals = b"".join(v for _, _, v in items) or b"\0"
        ko = np.cumsum([0] + [len(k) for k, _, _ in items[:-1]]).astype(np.uint64)
        vo = np.cumsum([0] + [len(v) for _, _, v in items[:-1]]).astype(np.uint64)
        kl = np.array([len(k) for k, _, _ in items], np.uint32)
        vs = np.array([len(v) for _, _, v in items], np.uint32)
        en = np.array([e for _, e, _ in items], np.uint8)
        out = ctypes.create_string_buffer(max_response + 16)
        kb, vb = ctypes.create_string_buffer(keys, len(keys)), ctypes.create_string_buffer(vals, len(vals))
        P = lambda a: ctypes.c_void_p(a.ctypes.data)
        r = self.f(kb, P(ko), P(kl), vb, P(vo), P(vs), P(en), len(items), elements,
                   max_response, maxrequestsize, 1 if reply_header else 0, out)
        return out.raw[:r] if r >= 0 else None


def reference():
    """The compiled reference codec, or None when oracle/_ref was not built."""
    if not os.path.exists(REF_SO):
        return None
    return _Codec(REF_SO, "ref_lzf_compress", "ref_lzf_decompress")
