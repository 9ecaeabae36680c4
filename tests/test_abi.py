"""The C-ABI boundary on CPU: the library builds, loads and exports every
symbol include/*.h declares; no compute call is made without a GPU."""
import ctypes
import os
import re

from tests.oracle_lib import ROOT, sha16, synth

import gibson_amd


def _declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b(lzf_\w+)\s*\(", src))


def test_headers_declare_the_reference_pair():
    # src/lzf.h:76-78, 95-97
    assert _declared("lzf.h") == {"lzf_compress", "lzf_decompress"}
    src = open(os.path.join(ROOT, "include", "lzf.h")).read()
    assert re.search(r"#define\s+LZF_VERSION\s+0x0105", src)
    assert 'extern "C"' in src


def _declared_gb():
    src = open(os.path.join(ROOT, "include", "gb_batch.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b(gb_\w+)\s*\(", src))


def test_library_exports_every_declared_symbol():
    L = gibson_amd.lib()
    for n in sorted(_declared_gb()):
        assert hasattr(L, n), n
    assert len(_declared_gb()) == 10
    names = _declared("lzf.h") | _declared("lzf_gpu.h")
    for n in sorted(names):
        assert hasattr(L, n), n
    assert set(gibson_amd.lzf.EXPORTS) <= names


def test_library_is_gfx950_code_object():
    data = open(gibson_amd.lib_path(), "rb").read()
    assert b"gfx950" in data


def test_no_cpu_codec_in_product_library():
    # the product library must not contain (or link) the oracle
    data = open(gibson_amd.lib_path(), "rb").read()
    assert b"oracle_lzf" not in data
    assert b"ref_lzf" not in data


def _kernels(path):
    # host-side stubs of the kernels a library can launch (nm of the .so)
    import subprocess
    out = subprocess.run(["nm", "-DC", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    return {m.group(1) for m in re.finditer(r"__device_stub__(?:void )?(\w+)", out)}


# the kernels the product routing launches, and nothing else
ROUTED = {"lzf_cand_stream_kernel", "lzf_parse_lane_kernel", "lzf_cand_table_kernel", "lzf_parse_rec_kernel",
          "lzf_compress_window_kernel", "lzf_decompress_pipe_kernel", "lzf_decompress_tokpar_kernel",
          "lzf_dsize_kernel", "lzf_lds_order_probe_kernel", "lzf_synth_kernel", "lzf_frame_size_kernel",
          "lzf_frame_scan_kernel", "lzf_frame_write_kernel", "lzf_frame_check_kernel",
          "lzf_move_kernel", "lzf_clear_tail_kernel"}
# cross-check forms: the diagnostic build only
DIAG_ONLY = {"lzf_wparse_kernel", "lzf_cand_q1_kernel", "lzf_cand_small_kernel", "lzf_cand_ring_kernel",
             "lzf_cand_mid_kernel", "lzf_compress_serial_kernel", "lzf_decompress_serial_kernel",
             "lzf_decompress_lane_kernel", "lzf_parse_wave_kernel"}


def test_product_library_holds_only_routed_kernels():
    prod = _kernels(gibson_amd.lib_path())
    assert prod == ROUTED, (sorted(prod - ROUTED), sorted(ROUTED - prod))
    data = open(gibson_amd.lib_path(), "rb").read()
    for name in ("lzf_launch_compress_wtab", "lzf_launch_cand_stream_rec", "lzf_launch_compress_serial"):
        assert name.encode() not in data, name
    diag = gibson_amd.lzf.diag_lib_path()
    if os.path.exists(diag):
        assert DIAG_ONLY <= _kernels(diag)


def test_version_constant():
    assert gibson_amd.LZF_VERSION == 0x0105


def test_host_generator_deterministic(golden):
    seen = 0
    for c in golden["compress"][:400]:
        assert sha16(synth(c["kind"], c["seed"], c["index"], c["n"])) == c["in_sha"]
        seen += 1
    assert seen


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    import importlib
    import gibson_amd.lzf as m
    monkeypatch.setattr(m, "_LIB", None)
    monkeypatch.setattr(m, "lib_path", lambda: str(tmp_path / "nope.so"))
    try:
        m.lib()
    except m.LzfLibraryMissing:
        pass
    else:
        raise AssertionError("missing library must raise")
    finally:
        importlib.reload(m)


def test_batch_calls_reject_bad_arguments_without_device():
    # argument validation happens before any HIP call, so this runs on CPU
    import ctypes
    L = gibson_amd.lib()
    null = ctypes.c_void_p(0)
    buf = ctypes.create_string_buffer(64)
    p = ctypes.cast(buf, ctypes.c_void_p)
    assert L.lzf_gpu_compress_batch(null, p, p, p, p, p, p, 1, 16, null) == -1
    assert L.lzf_gpu_compress_batch(p, p, p, p, p, p, p, 0, 16, null) == -1
    assert L.lzf_gpu_compress_batch(p, p, p, p, p, p, p, 1, (64 << 20) + 1, null) == -1
    assert L.lzf_gpu_decompress_batch(p, p, p, p, p, p, p, null, 1, 16, null) == -1
    assert L.lzf_gpu_decompress_batch(p, p, p, p, p, p, p, p, 0, 16, null) == -1
    assert L.lzf_gpu_synth_fill(0, 0, 0, 1, 0, 16, p, null) == -1
    assert L.lzf_host_compress_batch(null, p, p, p, p, p, p, 1) == -1
    assert L.lzf_host_decompress_batch(p, p, p, p, p, p, p, null, 0) == -1


def test_batch_calls_reject_bad_arguments_host_extensions():
    import ctypes
    L = gibson_amd.lib()
    null = ctypes.c_void_p(0)
    assert L.lzf_host_register(null, 64) == -1
    buf = ctypes.create_string_buffer(64)
    assert L.lzf_host_register(ctypes.cast(buf, ctypes.c_void_p), 0) == -1
    assert L.lzf_host_unregister(ctypes.cast(buf, ctypes.c_void_p)) == -1     # never registered
    assert L.lzf_host_decoded_size_batch(null, null, null, null, null, 0, 16) == -1
