"""ctypes mirror of liblzf_hip.so (include/lzf.h, include/lzf_gpu.h).

Names, argument meaning and error behaviour follow the reference API:
``lzf_compress(in, out_len)`` returns the stream or ``None`` (the C call's 0,
src/lzf_c.c:131/176/263/276); ``lzf_decompress(in, out_len)`` returns
``(bytes, 0)`` or ``(None, errno)`` with errno E2BIG / EINVAL in the order of
src/lzf_d.c:72-131.  There is no Python or CPU codec behind these names: a
missing or unloadable library raises ``LzfLibraryMissing``.
"""
import contextlib
import ctypes
import os

LZF_VERSION = 0x0105  # src/lzf.h:49

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

LZF_GPU_OK = 0
_ERRS = {-1: "EARG", -2: "ELAUNCH", -3: "ENODEV", -4: "ENOMEM"}

EXPORTS = (
    "lzf_compress",
    "lzf_decompress",
    "lzf_gpu_compress_batch",
    "lzf_gpu_decompress_batch",
    "lzf_gpu_synth_fill",
    "lzf_host_compress_batch",
    "lzf_host_decompress_batch",
    "lzf_gpu_kernel_info",
    "lzf_gpu_kv_frame_work_size",
    "lzf_gpu_kv_frame",
    "lzf_gpu_release",
    "lzf_host_register",
    "lzf_host_unregister",
    "lzf_gpu_device_plan",
    "lzf_host_last_spread",
    "lzf_host_split",
    "lzf_host_split_block",
    "lzf_host_split_policy",
    "lzf_gpu_parse_device_list",
)

# item encodings (src/net.h:274-278) and the MGET reply code (src/query.h:71)
ENC_PLAIN, ENC_LZF, ENC_NUMBER, ENC_NULL = 0x00, 0x01, 0x02, 0xFF
REPL_KVAL = 7


class LzfLibraryMissing(ImportError):
    pass


def lib_path():
    return os.path.join(_HERE, "liblzf_hip.so")


def diag_lib_path():
    """The diagnostic build (cross-check kernel forms; never the product)."""
    return os.path.join(_HERE, "liblzf_hip_diag.so")


_LOADED = {}


def lib():
    """Load liblzf_hip.so (built in-tree by __graft_entry__.build())."""
    global _LIB
    if _LIB is not None:
        return _LIB
    # LZF_HIP_LIB: load a diagnostic build (e.g. liblzf_hip_stats.so) instead
    _LIB = _load(os.environ.get("LZF_HIP_LIB") or lib_path())
    return _LIB


@contextlib.contextmanager
def using(path):
    """Route this module's calls through the library at ``path`` (e.g. the
    diagnostic build) for the duration of the block."""
    global _LIB
    prev = _LIB
    _LIB = _load(path)
    try:
        yield _LIB
    finally:
        _LIB = prev


def _load(path):
    if path in _LOADED:
        return _LOADED[path]
    if not os.path.exists(path):
        raise LzfLibraryMissing(f"{path} not built: run __graft_entry__.build() "
                                "(make -C gibson_amd/csrc); there is no CPU fallback")
    try:
        L = ctypes.CDLL(path, use_errno=True)
    except OSError as e:
        raise LzfLibraryMissing(f"cannot load {path}: {e}") from e
    u32, u64, vp, i32 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int32
    L.lzf_compress.restype = ctypes.c_uint
    L.lzf_compress.argtypes = [vp, ctypes.c_uint, vp, ctypes.c_uint]
    L.lzf_decompress.restype = ctypes.c_uint
    L.lzf_decompress.argtypes = [vp, ctypes.c_uint, vp, ctypes.c_uint]
    L.lzf_gpu_compress_batch.restype = ctypes.c_int
    L.lzf_gpu_compress_batch.argtypes = [vp, vp, vp, vp, vp, vp, vp, u32, u32, vp]
    L.lzf_gpu_decompress_batch.restype = ctypes.c_int
    L.lzf_gpu_decompress_batch.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, u32, u32, vp]
    L.lzf_gpu_synth_fill.restype = ctypes.c_int
    L.lzf_gpu_synth_fill.argtypes = [ctypes.c_int, u64, u64, u64, u32, u32, vp, vp]
    L.lzf_host_compress_batch.restype = ctypes.c_int
    L.lzf_host_compress_batch.argtypes = [vp, vp, vp, vp, vp, vp, vp, u32]
    L.lzf_host_decompress_batch.restype = ctypes.c_int
    L.lzf_host_decompress_batch.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, u32]
    L.lzf_gpu_release.restype = None
    L.lzf_gpu_release.argtypes = []
    L.lzf_gpu_kernel_info.restype = ctypes.c_char_p
    L.lzf_gpu_kernel_info.argtypes = []
    L.lzf_gpu_selfcheck.restype = ctypes.c_int
    L.lzf_gpu_selfcheck.argtypes = []
    L.lzf_gpu_lds_order_probe.restype = ctypes.c_int
    L.lzf_gpu_lds_order_probe.argtypes = []
    L.lzf_gpu_decoded_size_batch.restype = ctypes.c_int
    L.lzf_gpu_decoded_size_batch.argtypes = [vp, vp, vp, vp, vp, u32, u32, vp]
    L.lzf_host_decoded_size_batch.restype = ctypes.c_int
    L.lzf_host_decoded_size_batch.argtypes = [vp, vp, vp, vp, vp, u32, u32]
    L.lzf_gpu_kv_frame_work_size.restype = u64
    L.lzf_gpu_kv_frame_work_size.argtypes = [u32]
    L.lzf_gpu_kv_frame.restype = ctypes.c_int
    L.lzf_gpu_kv_frame.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, u32, u32, u32, ctypes.c_int,
                                   vp, u64, vp, vp, vp]
    L.lzf_host_register.restype = ctypes.c_int
    L.lzf_host_register.argtypes = [vp, u64]
    L.lzf_host_unregister.restype = ctypes.c_int
    L.lzf_host_unregister.argtypes = [vp]
    L.lzf_gpu_device_plan.restype = ctypes.c_int
    L.lzf_gpu_device_plan.argtypes = [vp, vp, vp, ctypes.c_int]
    L.lzf_host_last_spread.restype = ctypes.c_int
    L.lzf_host_last_spread.argtypes = [vp, vp, ctypes.c_int]
    L.lzf_host_split.restype = u32
    L.lzf_host_split.argtypes = [u32, u32, u32, vp, vp]
    L.lzf_host_split_block.restype = u32
    L.lzf_host_split_block.argtypes = [u32, u32, u32, vp]
    L.lzf_host_split_policy.restype = ctypes.c_int
    L.lzf_host_split_policy.argtypes = []
    L.lzf_gpu_parse_device_list.restype = ctypes.c_int
    L.lzf_gpu_parse_device_list.argtypes = [ctypes.c_char_p, ctypes.c_int, vp, ctypes.c_int]
    del i32
    _LOADED[path] = L
    return L


def selfcheck():
    """lzf_gpu_selfcheck(): 1 when the lane-ordered LDS exchange held on the
    current device, 0 when compress batches fall back to window64."""
    return int(lib().lzf_gpu_selfcheck())


def lds_order_probe():
    """lzf_gpu_lds_order_probe(): mismatching lanes of a fresh probe run."""
    return int(lib().lzf_gpu_lds_order_probe())


def decoded_size_batch(inp, in_off, in_len, out_size, err, out_limit, stream=None):
    """Device pre-pass: out_size/err of lzf_decompress at out_len = out_limit."""
    _check(lib().lzf_gpu_decoded_size_batch(_ptr(inp), _ptr(in_off), _ptr(in_len), _ptr(out_size), _ptr(err),
                                            int(in_off.numel()), int(out_limit), _stream_handle(stream)),
           "lzf_gpu_decoded_size_batch")


def kernel_info():
    return lib().lzf_gpu_kernel_info().decode()


def release():
    """lzf_gpu_release(): free the device scratch and this thread's staging."""
    lib().lzf_gpu_release()


def _check(rc, what):
    if rc != LZF_GPU_OK:
        raise RuntimeError(f"{what} failed: {_ERRS.get(rc, rc)}")


# ---- single-call drop-in (src/lzf.h:76-97) -------------------------------

def lzf_compress(data, out_len):
    """Compress ``data`` into at most ``out_len`` bytes; None if it does not fit."""
    data = bytes(data)
    src = ctypes.create_string_buffer(data, max(len(data), 1))
    dst = ctypes.create_string_buffer(max(out_len, 1))
    r = lib().lzf_compress(src, len(data), dst, out_len)
    return dst.raw[:r] if r else None


def lzf_decompress(data, out_len):
    """Decode ``data``; returns (bytes, 0) or (None, errno)."""
    data = bytes(data)
    # the reference reads one control byte even when in_len == 0
    src = ctypes.create_string_buffer(data + b"\xff", len(data) + 1)
    dst = ctypes.create_string_buffer(max(out_len, 1))
    ctypes.set_errno(0)
    r = lib().lzf_decompress(src, len(data), dst, out_len)
    if r:
        return dst.raw[:r], 0
    return None, ctypes.get_errno()


# ---- device batches over torch tensors -------------------------------------

def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def _stream_handle(stream):
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


def compress_batch(inp, in_off, in_len, out, out_off, out_cap, out_len, max_in_len, stream=None):
    """Device batch compress; all tensors on the same CUDA (HIP) device.
    inp/out uint8, *_off int64, in_len/out_cap/out_len int32 (read as u32)."""
    n = in_len.numel()
    rc = lib().lzf_gpu_compress_batch(_ptr(inp), _ptr(in_off), _ptr(in_len), _ptr(out),
                                      _ptr(out_off), _ptr(out_cap), _ptr(out_len), n,
                                      int(max_in_len), _stream_handle(stream))
    _check(rc, "lzf_gpu_compress_batch")


def decompress_batch(inp, in_off, in_len, out, out_off, out_cap, out_len, err, max_out_cap,
                     stream=None):
    n = in_len.numel()
    rc = lib().lzf_gpu_decompress_batch(_ptr(inp), _ptr(in_off), _ptr(in_len), _ptr(out),
                                        _ptr(out_off), _ptr(out_cap), _ptr(out_len), _ptr(err),
                                        n, int(max_out_cap), _stream_handle(stream))
    _check(rc, "lzf_gpu_decompress_batch")


def synth_fill(kind, seed, first, stride, count, n, out, stream=None):
    rc = lib().lzf_gpu_synth_fill(int(kind), int(seed), int(first), int(stride), int(count),
                                  int(n), _ptr(out), _stream_handle(stream))
    _check(rc, "lzf_gpu_synth_fill")


def _np_ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def host_compress_batch(inp, in_off, in_len, out, out_off, out_cap, out_len):
    """Host-memory batch (numpy arrays): PCIe staging inside the library."""
    rc = lib().lzf_host_compress_batch(_np_ptr(inp), _np_ptr(in_off), _np_ptr(in_len),
                                       _np_ptr(out), _np_ptr(out_off), _np_ptr(out_cap),
                                       _np_ptr(out_len), len(in_len))
    _check(rc, "lzf_host_compress_batch")


def host_decompress_batch(inp, in_off, in_len, out, out_off, out_cap, out_len, err):
    rc = lib().lzf_host_decompress_batch(_np_ptr(inp), _np_ptr(in_off), _np_ptr(in_len),
                                         _np_ptr(out), _np_ptr(out_off), _np_ptr(out_cap),
                                         _np_ptr(out_len), _np_ptr(err), len(in_len))
    _check(rc, "lzf_host_decompress_batch")


def host_register(arr):
    """lzf_host_register over a numpy array's bytes: the host batches whose
    arenas lie in registered ranges move values without CPU copies."""
    _check(lib().lzf_host_register(_np_ptr(arr), arr.nbytes), "lzf_host_register")


def host_unregister(arr):
    _check(lib().lzf_host_unregister(_np_ptr(arr)), "lzf_host_unregister")


def device_plan():
    """[(device, numa_node, bound)] of the host-memory calls (LZF_GPU_DEVICES)."""
    d, n, b = (ctypes.c_int * 64)(), (ctypes.c_int * 64)(), (ctypes.c_int * 64)()
    g = lib().lzf_gpu_device_plan(d, n, b, 64)
    if g < 0:
        raise RuntimeError(f"lzf_gpu_device_plan failed: {_ERRS.get(g, g)}")
    return [(d[k], n[k], bool(b[k])) for k in range(g)]


def host_last_spread():
    """[(values, ms)] per plan entry of this thread's last host-memory call."""
    v, t = (ctypes.c_uint32 * 64)(), (ctypes.c_double * 64)()
    g = lib().lzf_host_last_spread(v, t, 64)
    return [(v[k], t[k]) for k in range(min(g, 64))]


def host_split(count, groups, g):
    """(first, stride, n): the values entry g of ``groups`` takes."""
    f, s = ctypes.c_uint32(), ctypes.c_uint32()
    n = lib().lzf_host_split(count, groups, g, ctypes.byref(f), ctypes.byref(s))
    return f.value, s.value, n


def host_split_block(count, groups, g):
    """(first, n): the contiguous span entry g of ``groups`` takes under
    LZF_GPU_SPLIT=block."""
    f = ctypes.c_uint32()
    n = lib().lzf_host_split_block(count, groups, g, ctypes.byref(f))
    return f.value, n


def host_split_policy():
    """"block" when LZF_GPU_SPLIT=block is in force, else "round-robin"."""
    return "block" if lib().lzf_host_split_policy() == 1 else "round-robin"


def parse_device_list(spec, visible):
    out = (ctypes.c_int * 64)()
    n = lib().lzf_gpu_parse_device_list(spec.encode(), visible, out, 64)
    return list(out[:n]) if n > 0 else n


def kv_frame(keys, key_off, key_len, vals, val_off, val_size, enc, val_len, elements,
             max_val_len, frame, max_response, frame_len, work=None, reply_header=True,
             stream=None):
    """MGET / KEYS reply (src/net.c:1256-1342, header src/net.c:1162-1205)
    built on the device, LZF items decoded in place.  Tensors on one device:
    keys/vals/enc/frame uint8, *_off int64, key_len/val_size/val_len int32,
    frame_len int64 (1 element; 0 = CHECK_SPACE failed or an item did not
    decode to its val_len).  ``work`` defaults to a fresh scratch tensor."""
    import torch
    n = key_len.numel()
    if work is None:
        work = torch.empty(int(lib().lzf_gpu_kv_frame_work_size(n)), dtype=torch.uint8,
                           device=frame.device)
    rc = lib().lzf_gpu_kv_frame(_ptr(keys), _ptr(key_off), _ptr(key_len), _ptr(vals),
                                _ptr(val_off), _ptr(val_size), _ptr(enc), _ptr(val_len), n,
                                int(elements), int(max_val_len), 1 if reply_header else 0,
                                _ptr(frame), int(max_response), _ptr(frame_len), _ptr(work),
                                _stream_handle(stream))
    _check(rc, "lzf_gpu_kv_frame")
