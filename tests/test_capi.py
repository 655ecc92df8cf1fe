"""The C-ABI library: loads, exports every entry point include/*.h declares, host-side argument
checks. No compute here (CPU container) — the GPU tests drive the kernels."""
import ctypes
import os
import subprocess

import pytest


def test_library_exports_every_header_symbol(hc):
    names = hc.header_symbols()
    assert "hc_compress" in names and "hc_decompress_batch" in names and "hc_synth_batch" in names
    L = hc.lib()
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", hc.LIB_PATH], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(names) <= exported


def test_version_and_bound(hc):
    assert "gfx950" in hc.version()
    # worst case: runs of exactly three bytes expand RLE by 4/3
    assert hc.compress_bound(0) >= 9
    assert hc.compress_bound(262144) >= 9 + (262144 * 4 // 3) * 41 // 8


def test_host_side_status_without_device(hc):
    """Statuses decided before any device work match the reference's exit codes."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("host without GPU only")
    assert hc.compress(b"abc", width=0)[0] == hc.HC_ERR_WIDTH
    assert hc.compress(b"abcde", use_adapt=True, width=2)[0] == hc.HC_ERR_MATRIX_SIZE
    assert hc.compress(bytes(49), use_adapt=True, width=7)[0] == hc.HC_ERR_DIMS
    assert hc.decompress(b"12345678")[0] == hc.HC_ERR_HEADER
    # needs the device: fails loudly instead of falling back to the CPU
    assert hc.compress(b"abc")[0] == hc.HC_ERR_DEVICE
    assert hc.decompress(bytes(9))[0] == hc.HC_ERR_DEVICE


def test_batch_argument_validation(hc):
    L = hc.lib()
    null = ctypes.c_void_p(0)
    assert L.hc_compress_batch(null, null, null, 0, 0, null, null, null, null, null, null) == 0
    assert L.hc_compress_batch(null, null, null, 1, 0, null, null, null, null, null, null) == hc.HC_ERR_ARG
    one = ctypes.c_void_p(16)
    assert L.hc_compress_batch(one, one, one, 1, 0x40, one, one, one, one, one, null) == hc.HC_ERR_ARG
    odd = ctypes.c_void_p(17)
    assert L.hc_decompress_batch(odd, one, one, 1, one, one, one, one, one, null) == hc.HC_ERR_ARG


def test_headers_compile_as_c(hc, tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "hcodec.h"\n#include "hcodec_synth.h"\nint main(void){return HC_OK;}\n')
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", hc.INCLUDE_DIR, str(src), "-o",
                    str(tmp_path / "t")], check=True)


def test_shipping_library_has_no_hooks(hc):
    """The test / diagnostic hooks (hc_debug_*: forced tree layouts and encoder modes, shrunk
    buffer windows, traces, the adaptive stage clock) live in libhcodec_dbg.so only: the shipping
    libhcodec.so exports none of them and carries none of their global variables, so its entry
    points keep hcodec.h's "no hidden global state" (the reference: one HuffTree per call,
    transform.cpp:366,388)."""
    def syms(path, flags):
        out = subprocess.run(["nm", "-C", *flags, path], capture_output=True, text=True, check=True).stdout
        return out
    ship = syms(hc.LIB_PATH, ["-D", "--defined-only"])
    assert "hc_debug" not in ship
    allsyms = syms(hc.LIB_PATH, [])
    for g in ("g_window", "g_min_tree", "g_enc_tab", "g_trace", "g_clock"):
        assert g not in allsyms, g
    dbg = syms(hc.DBG_LIB_PATH, ["-D", "--defined-only"])
    for f in ("hc_debug_set_window", "hc_debug_set_min_tree", "hc_debug_set_enc_tab", "hc_debug_stage_clock",
              "hc_debug_stage_times", "hc_debug_set_trace"):
        assert f in dbg, f
    with pytest.raises(hc.HCodecError):  # hooks refuse to run against the shipping build
        hc.debug_set_min_tree(1)


def test_adapt_batch_rejects_short_workspace(hc):
    """hc_*_adapt_batch check work_bytes against the workspace's fixed part before any device
    work (a short workspace would otherwise be written out of bounds)"""
    L = hc.lib()
    one = ctypes.c_void_p(256)
    need = int(L.hc_adapt_compress_work_bound(0, 4))
    assert L.hc_compress_adapt_batch(one, one, one, one, 4, 0, one, one, one, one, one, one, need - 1,
                                     ctypes.c_void_p(0)) == hc.HC_ERR_ARG
    need = int(L.hc_adapt_decompress_work_bound(0, 0, 4))
    assert L.hc_decompress_adapt_batch(one, one, one, 4, one, one, one, one, one, one, need - 1,
                                       ctypes.c_void_p(0)) == hc.HC_ERR_ARG
