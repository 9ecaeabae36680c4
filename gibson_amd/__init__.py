"""gibson_amd -- MI355X-native LZF value codec for the Gibson cache server.

The product is the C-ABI library ``gibson_amd/liblzf_hip.so`` (include/lzf.h
drop-in + include/lzf_gpu.h batch API).  This package is the thin Python
mirror of that boundary used by bench.py and the tests: ctypes bindings with
the reference's names and semantics (``lzf_compress`` / ``lzf_decompress``,
src/lzf.h:76-97) plus device-batch helpers over torch tensors (torch is only
device-memory and stream plumbing here).
"""
from .lzf import (  # noqa: F401
    ENC_LZF,
    ENC_NULL,
    ENC_NUMBER,
    ENC_PLAIN,
    LZF_VERSION,
    REPL_KVAL,
    LzfLibraryMissing,
    compress_batch,
    decompress_batch,
    decoded_size_batch,
    lds_order_probe,
    selfcheck,
    kernel_info,
    release,
    lib,
    lib_path,
    lzf_compress,
    lzf_decompress,
    synth_fill,
    host_compress_batch,
    host_decompress_batch,
    host_register,
    host_unregister,
    device_plan,
    host_last_spread,
    host_split,
    host_split_block,
    host_split_policy,
    parse_device_list,
    kv_frame,
)
