"""GPU parity of the small-alphabet kernels -- the encoder's (hc_fgk.hip encode_kernel<.., kSmall>, the
small steps of its code_all_batch; model: tests/fgk_batch_model.py small_len, checked against the
one-symbol loop in tests/test_batch_model.py): while a stream has seen at most 16 symbols, up to
15 cached symbols of depth <= 4 are coded per step with exact leader tests from membership marks.
Streams whose MNP-5 symbols (transform.cpp:241-279) stay within a few values -- gradients,
two-level images, runs over a handful of bytes with a handful of lengths, exact ties -- and streams
whose alphabet grows past 16 partway (the steps hand over to the regular batches): in the
small-alphabet kernel forced on every stream, in the path-cache kernel, and through the automatic
vote (enc_mode_kernel sends a stream whose sample has at most 4 distinct run-start bytes to the
small kernel), with and without the diff model, byte for byte against the oracle
(transform.cpp:363-384, huffman.cpp:95-217), then decoded back -- by the decoder's small-alphabet
launch (decode_kernel<0, .., true>, Dec::decode_small: the same steps read back from the level
tables; chosen by payload rate under 2.5 bits per symbol, or forced for every narrow stream) and by
the regular one."""
import numpy as np
import pytest

from gpu_batch import compress_batch, decompress_batch

pytestmark = pytest.mark.gpu


def _streams(oracle_mod):
    rng = np.random.default_rng(23)
    raws = [oracle_mod.synth("grad", k, 512, 128 + 64 * k).tobytes() for k in range(6)]
    # two-level "images": runs of 0 / 255 with lengths from a small set
    for k in range(6):
        lens = rng.choice([3, 4, 7, 20, 258, 300][: 2 + k % 5], 2000)
        vals = np.resize(np.array([0, 255], np.uint8), lens.size)
        raws.append(np.repeat(vals, lens).tobytes())
    # a handful of byte values, a handful of run lengths
    for n_val in (2, 3, 4, 6):
        vals = rng.choice(256, n_val, replace=False).astype(np.uint8)
        lens = rng.choice([1, 2, 3, 5, 9, 258, 517], 4000, p=[0.3, 0.2, 0.2, 0.1, 0.1, 0.05, 0.05])
        raws.append(np.repeat(rng.choice(vals, lens.size), lens).tobytes())
    # exact ties: four values in lockstep (every update ties with its neighbours)
    raws.append(bytes([1, 2, 3, 4] * 5000))
    raws.append(bytes([9, 9, 9, 7, 7, 7] * 3000))
    # the alphabet grows past 16 partway: small steps first, then the regular batches
    grow = b"".join(bytes([v]) * (3 + v % 7) for v in range(40)) * 40
    raws.append(bytes([5, 5, 5, 6] * 4000) + grow + bytes([5, 5, 5, 6] * 4000))
    # ... and a photo (never small after its first symbols)
    raws.append(oracle_mod.synth("photo", 3, 256, 256).tobytes())
    return raws


def _decode_modes(hc, torch, encs, raws, modes=(0, 1, 2)):
    """every stream decoded back by each decoder launch choice (hc_debug_set_dec_small: 0 by rate,
    1 the small-alphabet launch for every narrow stream, 2 the regular launch for every one)"""
    hc.use_debug_build(True)
    try:
        for dm in modes:
            hc.debug_set_dec_small(dm)
            st, back, _ = decompress_batch(hc, torch, encs, [len(r) for r in raws])
            assert st == [0] * len(raws), dm
            for i, (r, b) in enumerate(zip(raws, back)):
                assert b == r, f"decoder mode {dm}, stream {i}"
    finally:
        hc.debug_set_dec_small(0)
        hc.use_debug_build(False)


@pytest.mark.parametrize("mode", [3, 1, 0], ids=["small", "cache", "vote"])
@pytest.mark.parametrize("use_diff", [True, False], ids=["cm", "c"])
def test_small_alphabet_steps_vs_oracle(gpu, hc, oracle_mod, use_diff, mode):
    torch = gpu
    raws = _streams(oracle_mod)
    hc.use_debug_build(True)
    try:
        hc.debug_set_enc_tab(mode)  # 3: the small-alphabet kernel for every stream, 1: the path cache
        st, encs, _ = compress_batch(hc, torch, raws, use_diff)
    finally:
        hc.debug_set_enc_tab(0)
        hc.use_debug_build(False)
    assert st == [0] * len(raws)
    for i, (r, e) in enumerate(zip(raws, encs)):
        want = oracle_mod.compress(r, use_diff, False, 512)
        assert want[0] == 0 and e == want[1], f"stream {i} ({len(r)} bytes)"
    # the shipping library's own choice, then each launch forced
    st, back, _ = decompress_batch(hc, torch, encs, [len(r) for r in raws])
    assert st == [0] * len(raws)
    assert [i for i, (r, b) in enumerate(zip(raws, back)) if r != b] == []
    if mode == 0:
        _decode_modes(hc, torch, encs, raws)


def test_small_alphabet_decoder_window_edges(gpu, hc, oracle_mod):
    """decode_small's steps across the input window's edges and the 256-symbol block ends: the
    grad / two-level streams under a 4 KB descriptor window, every narrow stream on the
    small-alphabet launch"""
    torch = gpu
    raws = _streams(oracle_mod)[:12]
    encs = [oracle_mod.compress(r, True, False, 512)[1] for r in raws]
    hc.use_debug_build(True)
    try:
        hc.debug_set_window(4096)
        for dm in (1, 2):
            hc.debug_set_dec_small(dm)
            st, back, _ = decompress_batch(hc, torch, encs, [len(r) for r in raws])
            assert st == [0] * len(raws), dm
            assert [i for i, (r, b) in enumerate(zip(raws, back)) if r != b] == [], dm
    finally:
        hc.debug_set_window(1 << 30)
        hc.debug_set_dec_small(0)
        hc.use_debug_build(False)


def test_small_alphabet_decoder_damaged_streams(gpu, hc, oracle_mod):
    """truncated and bit-flipped low-rate streams: the small-alphabet launch ends each with the
    oracle's status (the regular launch's, transform.cpp:394-398) and never runs past its buffers"""
    torch = gpu
    raws = _streams(oracle_mod)[:8]
    encs = [oracle_mod.compress(r, True, False, 512)[1] for r in raws]
    bad = []
    for k, e in enumerate(encs):
        bad.append(e[: len(e) // 2])  # truncated: count says more symbols than the payload holds
        b = bytearray(e)
        b[9 + (k * 131) % (len(e) - 9)] ^= 0x5A  # a flipped payload byte
        bad.append(bytes(b))
    wants = [oracle_mod.decompress(blob) for blob in bad]
    # capacity: the oracle's output exactly (a status-0 stream), or room to spare (an error
    # status outranks the capacity check, HcStatus)
    caps = [len(w[1]) if w[0] == 0 else 2 * len(raws[j // 2]) + 1024 for j, w in enumerate(wants)]
    res = {}
    hc.use_debug_build(True)
    try:
        for dm in (1, 2):
            hc.debug_set_dec_small(dm)
            res[dm] = decompress_batch(hc, torch, bad, caps)
    finally:
        hc.debug_set_dec_small(0)
        hc.use_debug_build(False)
    for j, want in enumerate(wants):
        for dm in (1, 2):
            st, back, _ = res[dm]
            assert st[j] == want[0], (dm, j)
            if want[0] == 0:
                assert back[j] == want[1], (dm, j)


def test_small_alphabet_grad_batch_digests(gpu, hc, oracle_mod):
    """the shipping library (no debug hooks) on the bench's grad batch shape: the reference's
    digests of grad k = 0..3 (512x512 -c -m) and a round trip of 256 streams"""
    import hashlib
    import json
    import os
    torch = gpu
    digests = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "digests.json")))
    raws = [oracle_mod.synth("grad", k, 512, 512).tobytes() for k in range(4)]
    st, encs, _ = compress_batch(hc, torch, raws, True)
    assert st == [0] * 4
    for k, e in enumerate(encs):
        want = digests["synthetic"][f"grad_{k}"]["cm"]
        assert (len(e), hashlib.sha256(e).hexdigest()) == (want["len"], want["sha256"]), k
    raws = [oracle_mod.synth("grad", k, 512, 512).tobytes() for k in range(200, 456)]
    st, encs, _ = compress_batch(hc, torch, raws, True)
    assert st == [0] * len(raws)
    st, back, _ = decompress_batch(hc, torch, encs, [len(r) for r in raws])
    assert st == [0] * len(raws)
    assert [i for i, (r, b) in enumerate(zip(raws, back)) if r != b] == []
    _decode_modes(hc, torch, encs[:32], raws[:32], (1, 2))
    for k in (0, 77, 255):
        assert encs[k] == oracle_mod.compress(raws[k], True, False, 512)[1]
