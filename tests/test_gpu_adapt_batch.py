"""GPU parity of the batched adaptive block RLE (hc_compress_adapt_batch /
hc_decompress_adapt_batch, through the C ABI) against the oracle and the reference's digests.

One batch mixes matrices that reach every kernel path: widths / heights that are not multiples
of 8 or of the 128-byte tile (edge blocks and partial tiles), matrices >= 256 on both sides
(block sizes 256 / 512 summed from tile summaries), flat and banded data (runs >= 258 in both
scan orders), photo and noise, with and without the diff model, plus the reference's error
cases (width 0 -> 4, size not a multiple of the width -> 6, a side < 8 -> 12).
Reference: transform.cpp:294-361, main.cpp:39-128.
"""
import hashlib
import random

import numpy as np
import pytest

from gpu_batch import compress_adapt_batch, decompress_adapt_batch

pytestmark = pytest.mark.gpu


def sha(b):
    return hashlib.sha256(b).hexdigest()


def _mat(oracle_mod, kind, w, h, seed):
    rng = random.Random(seed)
    if kind in ("photo", "noise", "grad"):
        return oracle_mod.synth(kind, seed, w, h).tobytes()
    if kind == "flat":
        return bytes([7]) * (w * h)
    if kind == "bands":
        return bytes(((y // 37) & 1) * 200 for y in range(h) for _ in range(w))
    out = bytearray()
    while len(out) < w * h:
        out += bytes([rng.randrange(3)]) * rng.randint(1, 300)
    return bytes(out[:w * h])


CASES = [("photo", 512, 512), ("photo", 136, 72), ("noise", 64, 200), ("flat", 300, 270),
         ("bands", 520, 264), ("runs", 129, 9), ("photo", 8, 8), ("grad", 257, 300), ("runs", 1000, 40),
         ("photo", 640, 16)]


@pytest.mark.parametrize("use_diff", [False, True])
def test_adapt_batch_vs_oracle(gpu, hc, oracle_mod, use_diff):
    torch = gpu
    raws = [_mat(oracle_mod, k, w, h, i) for i, (k, w, h) in enumerate(CASES)]
    widths = [w for _, w, _ in CASES]
    # error cases in the same batch: width 0, size not a multiple of the width, height < 8
    raws += [b"\x01" * 64, b"\x02" * 70, b"\x03" * 80]
    widths += [0, 8, 16]
    st, enc, _ = compress_adapt_batch(hc, torch, raws, widths, use_diff)
    for i, (r, w) in enumerate(zip(raws, widths)):
        want_st, want = oracle_mod.compress(r, use_diff, True, w) if w else (4, b"")
        assert st[i] == want_st, (i, st[i], want_st)
        if want_st == 0:
            assert enc[i] == want, f"matrix {i} {CASES[i]}: GPU adaptive stream differs from the oracle"
    ok = [i for i in range(len(raws)) if st[i] == 0]
    dst, dec, dlens = decompress_adapt_batch(hc, torch, [enc[i] for i in ok], [len(raws[i]) for i in ok])
    assert dst == [0] * len(ok)
    for j, i in enumerate(ok):
        assert dec[j] == raws[i], f"matrix {i}: round trip differs"


def test_adapt_batch_reference_digests(gpu, hc, oracle_mod, digests):
    """the reference's own -c -a / -c -a -m digests of the synthetic 512x512 streams, as one batch"""
    torch = gpu
    syn = digests["synthetic"]
    keys = sorted(k for k in syn if "ca" in syn[k] or "cma" in syn[k])
    raws = [oracle_mod.synth(k.rsplit("_", 1)[0], int(k.rsplit("_", 1)[1])).tobytes() for k in keys]
    for mode, d in (("ca", False), ("cma", True)):
        st, enc, _ = compress_adapt_batch(hc, torch, raws, [512] * len(raws), d)
        assert st == [0] * len(raws)
        for k, e in zip(keys, enc):
            assert (len(e), sha(e)) == (syn[k][mode]["len"], syn[k][mode]["sha256"]), (k, mode)
        dst, dec, _ = decompress_adapt_batch(hc, torch, enc, [len(r) for r in raws])
        assert dst == [0] * len(raws) and dec == raws


def test_adapt_batch_decode_errors_and_capacity(gpu, hc, oracle_mod, vectors):
    """malformed adaptive streams: the same status as the oracle (10 / 11 / 13 / 14 / 15 / 8 / 9);
    a short output capacity reports W * H"""
    torch = gpu
    blobs, want = [], []
    for v in vectors["decompress"]:
        b = bytes.fromhex(v["input"])
        if len(b) < 9 or not (b[8] & 0x40):
            continue
        blobs.append(b)
        want.append(v["rc"])
    assert sorted(set(want)) == [9, 10, 11, 13, 14, 15]
    r = oracle_mod.synth("photo", 3, 200, 100).tobytes()
    st0, good = oracle_mod.compress(r, True, True, 200)
    assert st0 == 0
    blobs += [good, good[:-3], good[:9] + b"\x00" * 3]
    want += [0, oracle_mod.decompress(good[:-3])[0], oracle_mod.decompress(good[:9] + b"\x00" * 3)[0]]
    caps = [1 << 20] * len(blobs)
    st, dec, lens = decompress_adapt_batch(hc, torch, blobs, caps)
    assert st == want
    st, _, lens = decompress_adapt_batch(hc, torch, [good], [len(r) - 1])
    assert st == [hc.HC_ERR_CAPACITY] and lens == [len(r)]


def _scaled(B, W, H, seed, noise):
    """constant B x B blocks of 3 values (the block size B wins), optionally with sparse noise
    that cuts every run below 259 (whole tiles then take tile_cost's counted path throughout)"""
    rng = np.random.default_rng(seed)
    v = rng.integers(0, 3, size=((H + B - 1) // B, (W + B - 1) // B)).astype(np.uint8)
    m = np.kron(v, np.ones((B, B), np.uint8))[:H, :W].copy()
    if noise:
        flat = m.reshape(-1)
        idx = rng.integers(0, flat.size, size=flat.size // 40)
        flat[idx] = rng.integers(0, 256, size=idx.size).astype(np.uint8)
    return m.tobytes()


@pytest.mark.parametrize("use_diff", [False, True])
def test_adapt_whole_tiles_each_block_size(gpu, hc, oracle_mod, use_diff):
    """whole 128 x 128 tiles where each candidate B = 8 .. 128 wins (blocks of that size), with
    runs of thousands (the monoid fallbacks of the counted costs) and cut by noise (the counted
    path): byte for byte the oracle, and the winning block sizes cover 8 .. 128"""
    torch = gpu
    raws, widths, won = [], [], set()
    for B in (8, 16, 32, 64, 128):
        for (W, H) in ((512, 512), (256, 384)):
            for noise in (False, True):
                pat = _scaled(B, W, H, B * 7 + W + noise, noise)
                r = bytes(oracle_mod.undiff(pat)) if use_diff else pat  # the diff model sees pat
                raws.append(r)
                widths.append(W)
                st = oracle_mod.adapt(pat, W, H)
                st = st[1] if isinstance(st, tuple) else st
                won.add(int.from_bytes(bytes(st[16:24]), "big"))
    assert {8, 16, 32, 64, 128} <= won
    st, enc, _ = compress_adapt_batch(hc, torch, raws, widths, use_diff)
    assert st == [0] * len(raws)
    for i, (r, w) in enumerate(zip(raws, widths)):
        want_st, want = oracle_mod.compress(r, use_diff, True, w)
        assert want_st == 0 and enc[i] == want, f"matrix {i}: GPU adaptive stream differs from the oracle"
    dst, dec, _ = decompress_adapt_batch(hc, torch, enc, [len(r) for r in raws])
    assert dst == [0] * len(raws) and dec == raws


def test_stage_clock(gpu, hc, oracle_mod):
    """the diagnostic stage clock bench.py reads: every stage of both batched adaptive calls,
    in launch order, with non-negative times; off again afterwards (the calls unchanged)"""
    torch = gpu
    raws = [oracle_mod.synth("photo", k, 256, 256).tobytes() for k in range(4)]
    hc.use_debug_build(True)  # the clock exists in the debug build only
    hc.debug_stage_clock(True)
    try:
        st, enc, _ = compress_adapt_batch(hc, torch, raws, [256] * 4, True)
        enc_stages = hc.debug_stage_times()
        dst, dec, _ = decompress_adapt_batch(hc, torch, enc, [len(r) for r in raws])
        dec_stages = hc.debug_stage_times()
    finally:
        hc.debug_stage_clock(False)
    assert st == [0] * 4 and dst == [0] * 4 and dec == raws
    assert [n for n, _ in enc_stages] == ["enc_plan", "tile_cost", "big_cost", "choose", "emit_tile", "emit_big",
                                         "fgk_encode", "status_fix"]
    assert [n for n, _ in dec_stages] == ["dec_plan", "fgk_decode", "dec_header", "bounds", "par_fsm", "par_entry",
                                         "par_z", "par_scan", "par_walk", "par_fix", "unblock_tile",
                                         "unblock", "chunk_sum", "chunk_scan", "undiff", "dec_final"]
    assert all(ms >= 0 for _, ms in enc_stages + dec_stages)
    try:
        with pytest.raises(hc.HCodecError):
            hc.debug_stage_times()
    finally:
        hc.use_debug_build(False)
    with pytest.raises(hc.HCodecError):  # the shipping build has no hooks
        hc.debug_stage_clock(True)
