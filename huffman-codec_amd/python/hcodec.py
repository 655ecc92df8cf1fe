"""ctypes binding to libhcodec.so (include/hcodec.h, include/hcodec_synth.h).

Host-side mirror of the reference's buffer-level interface (huffCompress / huffDecompress,
src/main.cpp:39-128) plus the batched device entry points. Torch is used only for device memory
and streams (tensors are passed by data_ptr()). There is deliberately no CPU fallback: if the
shared library is missing, every call raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
# HC_LIB_PATH: another build of the same library (A/B timing of kernel variants in one run)
LIB_PATH = os.environ.get("HC_LIB_PATH") or os.path.join(PKG, "lib", "libhcodec.so")
# the same sources built with the test / diagnostic hooks (-DHC_DEBUG_HOOKS): the hc_debug_*
# entry points exist only there, so the shipping library carries no mutable global state
DBG_LIB_PATH = os.environ.get("HC_DBG_LIB_PATH") or os.path.join(PKG, "lib", "libhcodec_dbg.so")
CLI_PATH = os.path.join(PKG, "bin", "huffman-codec")
BATCH_CLI_PATH = os.path.join(PKG, "bin", "huffman-codec-batch")
INCLUDE_DIR = os.path.join(os.path.dirname(PKG), "include")

HC_OK = 0
HC_ERR_WIDTH = 4
HC_ERR_MATRIX_SIZE = 6
HC_ERR_HEADER = 8
HC_ERR_HUFFMAN = 9
HC_ERR_ADAPT_HEADER = 10
HC_ERR_ADAPT_DIRS = 11
HC_ERR_DIMS = 12
HC_ERR_BLOCK_DATA = 13
HC_ERR_BLOCK_EOF = 14
HC_ERR_LEFTOVER = 15
HC_ERR_CAPACITY = 64
HC_ERR_UNSUPPORTED = 65
HC_ERR_BLOCK_SIZE = 66
HC_ERR_TOO_LARGE = 67
HC_ERR_DEVICE = 70
HC_ERR_ARG = 71

HC_FLAG_DIFF = 0x80
HC_FLAG_ADAPT = 0x40

SYNTH = {"noise": 0, "grad": 1, "photo": 2}

_libs = {}           # path -> loaded library
_active = LIB_PATH   # the library every call below goes to (use_debug_build switches it)


class HCodecError(RuntimeError):
    pass


def build():
    import subprocess
    subprocess.run(["make", "-s", "-C", PKG], check=True)


def use_debug_build(on=True):
    """Route every later call of this module to libhcodec_dbg.so (on) or back to the shipping
    libhcodec.so (off). Tests that set a debug hook run their calls on the debug build; the two
    libraries are separate code objects, each with its own device state."""
    global _active
    _active = DBG_LIB_PATH if on else LIB_PATH
    return lib()


def lib():
    """The active library (libhcodec.so unless use_debug_build); raise if it has not been built
    (no fallback path exists)."""
    return _load(_active)


def _load(path):
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise HCodecError(f"{path} missing: build it with `make -C {PKG}`")
    # torch ships its own libamdhip64.so.7 (same soname as /opt/rocm's). Whichever loads first
    # serves the whole process; loading ours first leaves torch without a GPU. So let torch's
    # runtime load first and libhcodec.so binds to it: one HIP runtime, shared device pointers.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(path)
    u8p = ctypes.c_void_p
    u64 = ctypes.c_uint64
    vp = ctypes.c_void_p
    L.hc_compress_bound.argtypes = [u64, ctypes.c_int]
    L.hc_compress_bound.restype = u64
    L.hc_compress.argtypes = [u8p, u64, ctypes.c_int, ctypes.c_int, u64, u8p, u64,
                              ctypes.POINTER(u64)]
    L.hc_decompress.argtypes = [u8p, u64, u8p, u64, ctypes.POINTER(u64)]
    L.hc_decompress_alloc.argtypes = [u8p, u64, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(u64)]
    L.hc_free.argtypes = [vp]
    L.hc_compress_batch.argtypes = [vp, vp, vp, ctypes.c_uint32, ctypes.c_uint32, vp, vp, vp, vp,
                                    vp, vp]
    L.hc_compress_batch_aux.argtypes = [vp, vp, vp, ctypes.c_uint32, ctypes.c_uint32, vp, vp, vp, vp,
                                        vp, vp, vp]
    L.hc_decompress_batch.argtypes = [vp, vp, vp, ctypes.c_uint32, vp, vp, vp, vp, vp, vp]
    L.hc_compress_host_batch.argtypes = [vp, vp, ctypes.c_uint32, ctypes.c_uint32, vp, vp, vp, vp]
    L.hc_decompress_host_batch.argtypes = [vp, vp, ctypes.c_uint32, vp, vp, vp, vp]
    L.hc_compress_adapt_host_batch.argtypes = [vp, vp, vp, ctypes.c_uint32, ctypes.c_uint32, vp, vp, vp, vp]
    L.hc_adapt_compress_work_bound.argtypes = [u64, ctypes.c_uint32]
    L.hc_adapt_compress_work_bound.restype = u64
    L.hc_adapt_decompress_work_bound.argtypes = [u64, u64, ctypes.c_uint32]
    L.hc_adapt_decompress_work_bound.restype = u64
    L.hc_compress_adapt_batch.argtypes = [vp, vp, vp, vp, ctypes.c_uint32, ctypes.c_uint32, vp, vp, vp, vp, vp,
                                          vp, u64, vp]
    L.hc_decompress_adapt_batch.argtypes = [vp, vp, vp, ctypes.c_uint32, vp, vp, vp, vp, vp, vp, u64, vp]
    L.hc_pack_batch.argtypes = [vp, vp, vp, ctypes.c_uint32, vp, vp, vp]
    L.hc_version.restype = ctypes.c_char_p
    L.hc_device_ok.restype = ctypes.c_int
    L.hc_device_info.argtypes = [ctypes.c_char_p, u64]
    L.hc_device_info.restype = ctypes.c_int
    L.hc_synth_batch.argtypes = [ctypes.c_int, u64, ctypes.c_uint32, u64, u64, vp, u64, vp]
    _libs[path] = L
    return L


def _dbg():
    """the debug build, which must be the active one (a hook set there would otherwise not
    affect the calls that follow)"""
    if _active != DBG_LIB_PATH:
        raise HCodecError("debug hooks need use_debug_build(True) first")
    return lib()


def release_cached():
    """hc_release_cached: free the library's cached device / pinned buffers"""
    lib().hc_release_cached()


def _buf(data):
    b = bytes(data)
    return b, ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p) if b else None


def compress(data, use_diff=False, use_adapt=False, width=512):
    """hc_compress: (status, encoded bytes). Mirrors huffCompress (main.cpp:39-87)."""
    b, p = _buf(data)
    cap = lib().hc_compress_bound(len(b), int(bool(use_adapt)))
    out = ctypes.create_string_buffer(max(int(cap), 1))
    n = ctypes.c_uint64(0)
    st = lib().hc_compress(p, len(b), int(bool(use_diff)), int(bool(use_adapt)), width,
                           ctypes.cast(out, ctypes.c_void_p), cap, ctypes.byref(n))
    return st, (out.raw[:n.value] if st == 0 else b"")


def decompress(data):
    """hc_decompress_alloc: (status, decoded bytes). Mirrors huffDecompress (main.cpp:90-128)."""
    b, p = _buf(data)
    q = ctypes.c_void_p()
    n = ctypes.c_uint64(0)
    st = lib().hc_decompress_alloc(p, len(b), ctypes.byref(q), ctypes.byref(n))
    out = b""
    if st == 0:
        out = ctypes.string_at(q, n.value) if n.value else b""
    if q:
        lib().hc_free(q)
    return st, out


def _stream_handle(stream):
    if stream is None:
        import torch
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    if isinstance(stream, int):
        return ctypes.c_void_p(stream)
    return ctypes.c_void_p(stream.cuda_stream)


def _dp(t):
    return ctypes.c_void_p(t.data_ptr())


def _check_batch(inp, in_offs, in_lens, out, out_offs, out_caps, out_lens, status):
    """The batch entry points take raw device pointers: a CPU, non-contiguous or wrongly typed
    tensor would become an out-of-bounds device access, so reject it here instead."""
    import torch
    n = in_offs.numel()
    spec = (("in", inp, torch.uint8, None), ("in_offs", in_offs, torch.int64, n),
            ("in_lens", in_lens, torch.int64, n), ("out", out, torch.uint8, None),
            ("out_offs", out_offs, torch.int64, n), ("out_caps", out_caps, torch.int64, n),
            ("out_lens", out_lens, torch.int64, n), ("status", status, torch.int32, n))
    dev = inp.device
    for name, t, dt, numel in spec:
        if not isinstance(t, torch.Tensor):
            raise TypeError(f"{name}: expected a torch tensor")
        if not t.is_cuda or t.device != dev:
            raise ValueError(f"{name}: expected a CUDA tensor on {dev}, got {t.device}")
        if t.dtype != dt:
            raise TypeError(f"{name}: expected {dt}, got {t.dtype}")
        if not t.is_contiguous():
            raise ValueError(f"{name}: not contiguous")
        if numel is not None and t.numel() != numel:
            raise ValueError(f"{name}: {t.numel()} entries for {n} streams")
    return n


_AUX = {}  # device index -> a side stream for the encoder's table-mode launches (Python-side)


def _aux_stream(inp):
    import torch
    d = inp.device.index if inp.device.index is not None else torch.cuda.current_device()
    if d not in _AUX:
        _AUX[d] = torch.cuda.Stream(device=d)
    return _AUX[d]


def compress_batch(inp, in_offs, in_lens, out, out_offs, out_caps, out_lens, status,
                   use_diff=False, stream=None, aux_stream="auto"):
    """hc_compress_batch_aux on torch CUDA tensors (uint8 data, int64 offsets/lengths, int32
    status). aux_stream: a second stream for the table-mode launches ("auto": one side stream
    per device kept by this module; None: both modes one after the other on `stream`)."""
    n = _check_batch(inp, in_offs, in_lens, out, out_offs, out_caps, out_lens, status)
    aux = _aux_stream(inp) if aux_stream == "auto" else aux_stream
    rc = lib().hc_compress_batch_aux(_dp(inp), _dp(in_offs), _dp(in_lens), n,
                                     HC_FLAG_DIFF if use_diff else 0, _dp(out), _dp(out_offs),
                                     _dp(out_caps), _dp(out_lens), _dp(status), _stream_handle(stream),
                                     ctypes.c_void_p(None) if aux is None else _stream_handle(aux))
    if rc:
        raise HCodecError(f"hc_compress_batch failed: {rc}")


def decompress_batch(inp, in_offs, in_lens, out, out_offs, out_caps, out_lens, status, stream=None):
    """hc_decompress_batch on torch CUDA tensors (same layout as compress_batch)."""
    n = _check_batch(inp, in_offs, in_lens, out, out_offs, out_caps, out_lens, status)
    rc = lib().hc_decompress_batch(_dp(inp), _dp(in_offs), _dp(in_lens), n, _dp(out),
                                   _dp(out_offs), _dp(out_caps), _dp(out_lens), _dp(status),
                                   _stream_handle(stream))
    if rc:
        raise HCodecError(f"hc_decompress_batch failed: {rc}")


def _work(nbytes, device):
    import torch
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


def _check_work(work, device, need):
    import torch
    if not (isinstance(work, torch.Tensor) and work.is_cuda and work.device == device
            and work.dtype == torch.uint8 and work.is_contiguous()):
        raise ValueError(f"work: expected a contiguous uint8 CUDA tensor on {device}")
    if work.data_ptr() % 16:
        raise ValueError("work: must be 16-byte aligned")
    if work.numel() < need:
        raise ValueError(f"work: {work.numel()} bytes, the call needs {need}")


def compress_adapt_batch(inp, in_offs, in_lens, widths, out, out_offs, out_caps, out_lens, status,
                         use_diff=False, stream=None, work=None):
    """hc_compress_adapt_batch (-a, optionally -m) on CUDA tensors; widths: int64 per matrix.
    The workspace is allocated here unless given (uint8 CUDA tensor)."""
    n = _check_batch(inp, in_offs, in_lens, out, out_offs, out_caps, out_lens, status)
    _check_batch(inp, in_offs, widths, out, out_offs, out_caps, out_lens, status)
    need = int(lib().hc_adapt_compress_work_bound(int(in_lens.sum()), n))
    if work is None:
        work = _work(need, inp.device)
    _check_work(work, inp.device, need)
    rc = lib().hc_compress_adapt_batch(_dp(inp), _dp(in_offs), _dp(in_lens), _dp(widths), n,
                                       HC_FLAG_DIFF if use_diff else 0, _dp(out), _dp(out_offs), _dp(out_caps),
                                       _dp(out_lens), _dp(status), _dp(work), work.numel(),
                                       _stream_handle(stream))
    if rc:
        raise HCodecError(f"hc_compress_adapt_batch failed: {rc}")
    return work


def decompress_adapt_batch(inp, in_offs, in_lens, out, out_offs, out_caps, out_lens, status, stream=None,
                           work=None):
    """hc_decompress_adapt_batch on CUDA tensors (adaptive streams -> matrices)."""
    n = _check_batch(inp, in_offs, in_lens, out, out_offs, out_caps, out_lens, status)
    need = int(lib().hc_adapt_decompress_work_bound(int(in_lens.sum()), int(out_caps.sum()), n))
    if work is None:
        work = _work(need, inp.device)
    _check_work(work, inp.device, need)
    rc = lib().hc_decompress_adapt_batch(_dp(inp), _dp(in_offs), _dp(in_lens), n, _dp(out), _dp(out_offs),
                                         _dp(out_caps), _dp(out_lens), _dp(status), _dp(work), work.numel(),
                                         _stream_handle(stream))
    if rc:
        raise HCodecError(f"hc_decompress_adapt_batch failed: {rc}")
    return work


def pack_batch(inp, in_offs, lens, out, out_offs, stream=None):
    """hc_pack_batch on CUDA tensors: out[out_offs[i]:+lens[i]] = inp[in_offs[i]:+lens[i]]."""
    import torch
    n = in_offs.numel()
    for name, t, dt in (("in", inp, torch.uint8), ("in_offs", in_offs, torch.int64), ("lens", lens, torch.int64),
                        ("out", out, torch.uint8), ("out_offs", out_offs, torch.int64)):
        if not (isinstance(t, torch.Tensor) and t.is_cuda and t.device == inp.device and t.dtype == dt
                and t.is_contiguous()):
            raise ValueError(f"{name}: expected a contiguous {dt} CUDA tensor on {inp.device}")
    if lens.numel() != n or out_offs.numel() != n:
        raise ValueError("in_offs, lens and out_offs must have one entry per range")
    rc = lib().hc_pack_batch(_dp(inp), _dp(in_offs), _dp(lens), n, _dp(out), _dp(out_offs),
                             _stream_handle(stream))
    if rc:
        raise HCodecError(f"hc_pack_batch failed: {rc}")


def _host_batch(fn, blobs, caps, *extra):
    """blobs in host memory -> (statuses, outputs) through a host-batch entry point"""
    n = len(blobs)
    keep = [bytes(b) for b in blobs]
    ins = (ctypes.c_void_p * max(n, 1))(*[ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p) if b else None
                                          for b in keep])
    lens = (ctypes.c_uint64 * max(n, 1))(*[len(b) for b in keep])
    outs_buf = [ctypes.create_string_buffer(max(int(c), 1)) for c in caps]
    outs = (ctypes.c_void_p * max(n, 1))(*[ctypes.cast(o, ctypes.c_void_p) for o in outs_buf])
    ocaps = (ctypes.c_uint64 * max(n, 1))(*[int(c) for c in caps])
    olens = (ctypes.c_uint64 * max(n, 1))()
    st = (ctypes.c_int32 * max(n, 1))()
    rc = fn(ctypes.cast(ins, ctypes.c_void_p), ctypes.cast(lens, ctypes.c_void_p), n, *extra,
            ctypes.cast(outs, ctypes.c_void_p), ctypes.cast(ocaps, ctypes.c_void_p),
            ctypes.cast(olens, ctypes.c_void_p), ctypes.cast(st, ctypes.c_void_p))
    if rc:
        raise HCodecError(f"host batch failed: {rc}")
    res = [outs_buf[i].raw[:olens[i]] if st[i] == 0 else b"" for i in range(n)]
    return [st[i] for i in range(n)], res, [olens[i] for i in range(n)]


def compress_host_batch(blobs, use_diff=False, caps=None):
    """hc_compress_host_batch on host byte strings: (statuses, encoded, out_lens)."""
    caps = caps if caps is not None else [compress_bound(len(b)) for b in blobs]
    return _host_batch(lib().hc_compress_host_batch, blobs, caps, HC_FLAG_DIFF if use_diff else 0)


def compress_adapt_host_batch(blobs, widths, use_diff=False, caps=None):
    """hc_compress_adapt_host_batch on host byte strings (-a, one matrix of widths[i] per blob):
    (statuses, encoded, out_lens)."""
    caps = caps if caps is not None else [compress_bound(len(b), True) for b in blobs]
    w = (ctypes.c_uint64 * max(len(blobs), 1))(*[int(x) for x in widths])
    L = lib()

    def fn(ins, lens, n, outs, ocaps, olens, st):
        return L.hc_compress_adapt_host_batch(ins, lens, ctypes.cast(w, ctypes.c_void_p), n,
                                              HC_FLAG_DIFF if use_diff else 0, outs, ocaps, olens, st)
    return _host_batch(fn, blobs, caps)


def decompress_host_batch(blobs, caps):
    """hc_decompress_host_batch on host byte strings: (statuses, decoded, out_lens)."""
    return _host_batch(lib().hc_decompress_host_batch, blobs, caps)


def synth_batch(kind, k0, n_streams, width, height, out, stride, stream=None):
    """hc_synth_batch: SURVEY.md Appendix D inputs generated in device memory."""
    rc = lib().hc_synth_batch(SYNTH.get(kind, kind), k0, n_streams, width, height, _dp(out),
                              stride, _stream_handle(stream))
    if rc:
        raise HCodecError(f"hc_synth_batch failed: {rc}")


def debug_set_window(nbytes):
    """Test hook (debug build only, use_debug_build): the FGK kernels reach each stream through buffer
    windows that slide every `nbytes` (default 1 GiB); a small window makes ordinary streams
    cross many window edges. Affects every later launch in this process."""
    f = _dbg().hc_debug_set_window
    f.argtypes = [ctypes.c_uint32]
    rc = f(int(nbytes))
    if rc:
        raise HCodecError(f"hc_debug_set_window failed: {rc}")


def debug_set_min_tree(kind):
    """Test hook (debug build only, use_debug_build): the smallest FGK tree layout every later launch
    in this process may use (0 narrow, 1 wide, 2 huge: 64-bit weights), so that small streams
    exercise the kernels otherwise reserved for streams of > 2^22 - 2 / >= 2^32 - 1 symbols."""
    f = _dbg().hc_debug_set_min_tree
    f.argtypes = [ctypes.c_uint32]
    rc = f(int(kind))
    if rc:
        raise HCodecError(f"hc_debug_set_min_tree failed: {rc}")


def debug_set_enc_tab(mode):
    """Test hook (debug build only, use_debug_build): how the encoder finds a symbol's code for
    narrow / wide streams: 0 per stream from a sample of its alphabet (the default), 1 the path
    cache for every stream, 2 the level tables for every stream, 3 the small-alphabet kernel for
    every narrow stream."""
    f = _dbg().hc_debug_set_enc_tab
    f.argtypes = [ctypes.c_uint32]
    rc = f(int(mode))
    if rc:
        raise HCodecError(f"hc_debug_set_enc_tab failed: {rc}")


def debug_set_dec_small(mode):
    """Test hook (debug build only, use_debug_build): which decoder launch takes a narrow stream:
    0 by its payload rate (under 2.5 bits per symbol: the small-alphabet launch; the default), 1
    the small-alphabet launch for every one, 2 the regular launch for every one."""
    f = _dbg().hc_debug_set_dec_small
    f.argtypes = [ctypes.c_uint32]
    rc = f(int(mode))
    if rc:
        raise HCodecError(f"hc_debug_set_dec_small failed: {rc}")


def debug_enc_votes(inp, in_offs, in_lens, use_diff, low_occ, status, stream=None):
    """Test hook (debug build only, use_debug_build): the encoder's per-stream mode vote alone
    (enc_mode_kernel) into status: -0x7A1 the path cache, -0x7A0 the level tables. low_occ: the
    batch fits table mode's residency (what the launcher passes for <= 24 streams per CU)."""
    n = _check_batch(inp, in_offs, in_lens, inp, in_offs, in_lens, in_lens, status)
    f = _dbg().hc_debug_enc_votes
    f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint32] * 3 + [ctypes.c_void_p] * 2
    rc = f(_dp(inp), _dp(in_offs), _dp(in_lens), n, HC_FLAG_DIFF if use_diff else 0, 1 if low_occ else 0, _dp(status),
           _stream_handle(stream))
    if rc:
        raise HCodecError(f"hc_debug_enc_votes failed: {rc}")


def debug_set_par_min(symbols):
    """Test hook (debug build only, use_debug_build): adaptive streams of at least `symbols` block
    symbols find their block boundaries by the parallel pass (default 2^20; 0: every stream)."""
    f = _dbg().hc_debug_set_par_min
    f.argtypes = [ctypes.c_uint64]
    rc = f(int(symbols))
    if rc:
        raise HCodecError(f"hc_debug_set_par_min failed: {rc}")


def debug_set_par_skew(nbytes):
    """Test hook (debug build only, use_debug_build): every odd chunk of the parallel block-boundary
    pass walks from its predicted entry shifted by `nbytes` output bytes (0: off), forcing par_fix's
    re-runs and its repair of the block starts a wrong walk wrote."""
    f = _dbg().hc_debug_set_par_skew
    f.argtypes = [ctypes.c_uint64]
    rc = f(int(nbytes))
    if rc:
        raise HCodecError(f"hc_debug_set_par_skew failed: {rc}")


def debug_stage_clock(on):
    """Diagnostic (debug build only, use_debug_build): when on, the batched adaptive calls of
    this thread record a HIP event after each stage; debug_stage_times() reads the last call's."""
    f = _dbg().hc_debug_stage_clock
    f.argtypes = [ctypes.c_int]
    f(1 if on else 0)


def debug_stage_times():
    """[(stage, ms), ...] of the last batched adaptive call (waits for it); needs the clock on"""
    f = _dbg().hc_debug_stage_times
    f.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.c_int]
    names = ctypes.create_string_buffer(1024)
    ms = (ctypes.c_float * 32)()
    n = f(names, 1024, ms, 32)
    if n < 0:
        raise HCodecError("hc_debug_stage_times failed (clock off?)")
    return list(zip(names.value.decode().split("\n")[:n], [float(ms[k]) for k in range(n)]))


def compress_bound(n, use_adapt=False):
    return int(lib().hc_compress_bound(n, int(bool(use_adapt))))


def device_ok():
    return bool(lib().hc_device_ok())


def device_info():
    buf = ctypes.create_string_buffer(512)
    lib().hc_device_info(buf, 512)
    return buf.value.decode()


def version():
    return lib().hc_version().decode()


def header_symbols():
    """Every function name declared in include/*.h (the exported surface)."""
    import re
    names = []
    for fn in sorted(os.listdir(INCLUDE_DIR)):
        if fn.endswith(".h"):
            txt = open(os.path.join(INCLUDE_DIR, fn)).read()
            txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
            names += re.findall(r"\b(hc_[a-z0-9_]+)\s*\(", txt)
    return sorted(set(names))
