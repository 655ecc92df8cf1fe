"""ctypes wrapper around oracle/_build/liboracle.so (the C restatement, hc_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, and only as the checker. The product path never imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
REF_BIN = os.path.join(HERE, "_ref", "huffman-codec")
REF_BIN_O2 = os.path.join(HERE, "_ref", "huffman-codec-O2")

NOISE, GRAD, PHOTO = 0, 1, 2
KINDS = {"noise": NOISE, "grad": GRAD, "photo": PHOTO}

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE, "_build/liboracle.so"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        u64 = ctypes.c_uint64
        L.hco_compress.argtypes = [u8p, u64, ctypes.c_int, ctypes.c_int, u64,
                                   ctypes.POINTER(u8p), ctypes.POINTER(u64)]
        L.hco_decompress.argtypes = [u8p, u64, ctypes.POINTER(u8p), ctypes.POINTER(u64)]
        L.hco_free.argtypes = [ctypes.c_void_p]
        L.hco_synth.argtypes = [ctypes.c_int, u64, u64, u64, u8p]
        L.hco_rle_apply.argtypes = [u8p, u64, u8p]
        L.hco_rle_apply.restype = u64
        L.hco_rle_revert.argtypes = [u8p, u64, u8p, u64]
        L.hco_rle_revert.restype = u64
        L.hco_diff_apply.argtypes = [u8p, u64]
        L.hco_diff_revert.argtypes = [u8p, u64]
        L.hco_fgk_bound.argtypes = [u64]
        L.hco_fgk_bound.restype = u64
        for f in (L.hco_fgk_encode, L.hco_fgk_encode_slot):
            f.argtypes = [u8p, u64, u8p]
            f.restype = u64
        for f in (L.hco_fgk_decode, L.hco_fgk_decode_slot):
            f.argtypes = [u8p, u64, u64, u8p]
        L.hco_adapt_bound.argtypes = [u64, u64]
        L.hco_adapt_bound.restype = u64
        L.hco_adapt_apply.argtypes = [u8p, u64, u64, u8p, ctypes.POINTER(u64), ctypes.POINTER(u64)]
        L.hco_adapt_revert.argtypes = [u8p, u64, ctypes.POINTER(u8p), ctypes.POINTER(u64)]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def _u8(data):
    return np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8)) if not isinstance(
        data, np.ndarray) else np.ascontiguousarray(data, dtype=np.uint8)


def _take(p, n):
    out = bytes(ctypes.string_at(p, n.value)) if n.value else b""
    lib().hco_free(p)
    return out


def compress(data, use_diff=False, use_adapt=False, width=512):
    """huffCompress (main.cpp:39-87). Returns (status, bytes)."""
    a = _u8(data)
    p = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_uint64(0)
    st = lib().hco_compress(_ptr(a), a.size, int(use_diff), int(use_adapt), width,
                            ctypes.byref(p), ctypes.byref(n))
    if st:
        return st, b""
    return 0, _take(p, n)


def decompress(data):
    """huffDecompress (main.cpp:90-128). Returns (status, bytes)."""
    a = _u8(data)
    p = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_uint64(0)
    st = lib().hco_decompress(_ptr(a), a.size, ctypes.byref(p), ctypes.byref(n))
    if st:
        return st, b""
    return 0, _take(p, n)


def synth(kind, k, width=512, height=512):
    """SURVEY.md Appendix D generator; kind in {'noise','grad','photo'} or 0/1/2."""
    kind = KINDS.get(kind, kind)
    out = np.empty(width * height, dtype=np.uint8)
    lib().hco_synth(int(kind), k, width, height, _ptr(out))
    return out


def rle(data):
    a = _u8(data)
    out = np.empty(a.size + a.size // 3 + 8, dtype=np.uint8)
    n = lib().hco_rle_apply(_ptr(a), a.size, _ptr(out))
    return out[:n].tobytes()


def unrle(data):
    a = _u8(data)
    n = lib().hco_rle_revert(_ptr(a), a.size, None, 0)
    out = np.empty(max(n, 1), dtype=np.uint8)
    lib().hco_rle_revert(_ptr(a), a.size, _ptr(out), n)
    return out[:n].tobytes()


def diff(data):
    a = _u8(data).copy()
    lib().hco_diff_apply(_ptr(a), a.size)
    return a.tobytes()


def undiff(data):
    a = _u8(data).copy()
    lib().hco_diff_revert(_ptr(a), a.size)
    return a.tobytes()


def fgk_encode(symbols, slot_form=False):
    """Returns (payload bytes, bit count before padding)."""
    a = _u8(symbols)
    out = np.empty(lib().hco_fgk_bound(a.size), dtype=np.uint8)
    f = lib().hco_fgk_encode_slot if slot_form else lib().hco_fgk_encode
    nbits = f(_ptr(a), a.size, _ptr(out))
    return out[:(nbits + 7) // 8].tobytes(), nbits


def fgk_decode(payload, count, slot_form=False):
    a = _u8(payload)
    out = np.empty(max(count, 1), dtype=np.uint8)
    f = lib().hco_fgk_decode_slot if slot_form else lib().hco_fgk_decode
    st = f(_ptr(a), a.size * 8, count, _ptr(out))
    return st, out[:count].tobytes()


def adapt(matrix, width, height):
    """applyAdaptRLE (transform.cpp:294-328). Returns (status, stream, block size)."""
    a = _u8(matrix)
    out = np.empty(lib().hco_adapt_bound(a.size, width), dtype=np.uint8)
    n = ctypes.c_uint64(0)
    b = ctypes.c_uint64(0)
    st = lib().hco_adapt_apply(_ptr(a), width, height, _ptr(out), ctypes.byref(n), ctypes.byref(b))
    return st, out[:n.value].tobytes(), b.value


def unadapt(stream):
    a = _u8(stream)
    p = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_uint64(0)
    st = lib().hco_adapt_revert(_ptr(a), a.size, ctypes.byref(p), ctypes.byref(n))
    if st:
        return st, b""
    return 0, _take(p, n)


def ref_available(o2=False):
    return os.path.exists(REF_BIN_O2 if o2 else REF_BIN)


def run_ref(args, input_bytes, workdir, o2=False, timeout=None):
    """Run the compiled reference (oracle/_ref) on input_bytes. Returns (rc, output bytes, stderr)."""
    inp = os.path.join(workdir, "ref_in.bin")
    outp = os.path.join(workdir, "ref_out.bin")
    with open(inp, "wb") as f:
        f.write(input_bytes)
    if os.path.exists(outp):
        os.remove(outp)
    r = subprocess.run([REF_BIN_O2 if o2 else REF_BIN] + list(args) + ["-i", inp, "-o", outp],
                       capture_output=True, timeout=timeout)
    out = b""
    if os.path.exists(outp):
        with open(outp, "rb") as f:
            out = f.read()
    return r.returncode, out, r.stderr.decode(errors="replace")
