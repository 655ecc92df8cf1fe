"""GPU parity of the adaptive decoder's PARALLEL block-boundary pass (hc_adapt.hip par_fsm /
par_entry / par_z / par_scan / par_walk / par_fix; algorithm and argument:
tests/bounds_par_model.py) against the oracle, which runs the reference's serial process
(revertAdaptRLE transform.cpp:330-361 / revertRLEBlock transform.cpp:162-187).

  * the debug build's threshold lowered to 0 (hc_debug_set_par_min): every adaptive stream of
    the serial pass's own edge-case tests (tests/test_gpu_adaptive_bounds.py: ragged blocks,
    many blocks per step, zero counts, forged block sizes, narrow matrices, exit codes
    13 / 14 / 15) and the batched adaptive tests' matrices take the parallel pass;
  * the shipping build at its real threshold (2^20 block symbols): large matrices (photo
    2048 x 2048 with and without the diff model, a forged 8 x 8-block stream of constant runs)
    round-trip, and their damaged variants report the oracle's status.
"""
import numpy as np
import pytest

import test_gpu_adaptive_bounds as B
from gpu_batch import compress_adapt_batch, decompress_adapt_batch

pytestmark = pytest.mark.gpu


@pytest.fixture
def par_everywhere(gpu, hc):
    hc.use_debug_build(True)
    hc.debug_set_par_min(0)
    yield
    hc.debug_set_par_min(1 << 20)
    hc.use_debug_build(False)


def test_par_bounds_valid_and_corrupted(gpu, hc, oracle_mod, par_everywhere):
    B.test_bounds_valid_and_corrupted_vs_oracle(gpu, hc, oracle_mod)


def test_par_bounds_many_blocks_per_step(gpu, hc, oracle_mod, par_everywhere):
    B.test_bounds_many_blocks_per_step(gpu, hc, oracle_mod)


def test_par_bounds_other_block_sizes(gpu, hc, oracle_mod, par_everywhere):
    B.test_bounds_other_block_sizes_vs_oracle(gpu, hc, oracle_mod)


def test_par_bounds_narrow_forged(gpu, hc, oracle_mod, par_everywhere):
    B.test_bounds_narrow_forged_matrices_vs_oracle(gpu, hc, oracle_mod)


def test_par_bounds_batch_round_trip(gpu, hc, oracle_mod, par_everywhere):
    """encoder output (photo / noise / runs, both diff settings) decoded as one batch through the
    parallel pass: the oracle's encodings, decoded back to the inputs"""
    torch = gpu
    raws, widths = [], []
    for k, (kind, w, h) in enumerate([("photo", 512, 512), ("photo", 300, 170), ("noise", 96, 200),
                                      ("grad", 257, 300), ("photo", 64, 64)]):
        raws.append(oracle_mod.synth(kind, k, w, h).tobytes())
        widths.append(w)
    for use_diff in (False, True):
        st, enc, _ = compress_adapt_batch(hc, torch, raws, widths, use_diff)
        assert st == [0] * len(raws)
        for r, w, e in zip(raws, widths, enc):
            assert oracle_mod.compress(r, use_diff, True, w) == (0, e)
        dst, dec, _ = decompress_adapt_batch(hc, torch, enc, [len(r) for r in raws])
        assert dst == [0] * len(raws) and dec == raws


def _damaged(rng, x):
    """variants of a block-symbol list: truncated (14 or 13), extended (15), one symbol changed"""
    out = [x[: len(x) - int(rng.integers(1, 40))], x + [1, 2, 3]]
    for _ in range(2):
        y = list(x)
        k = int(rng.integers(0, len(y)))
        y[k] = (y[k] + int(rng.integers(1, 256))) & 255
        out.append(y)
    return out


def _adaptive_parts(oracle_mod, stream):
    st = np.frombuffer(stream, dtype=np.uint8)
    w, h, b = (int.from_bytes(st[8 * i:8 * i + 8].tobytes(), "big") for i in range(3))
    nb = -(-w // b) * -(-h // b)
    hdr = 24 + -(-nb // 8)
    return list(st[:hdr].tobytes()), st[hdr:].tolist()


@pytest.mark.parametrize("use_diff", [False, True])
def test_par_bounds_real_threshold_photo(gpu, hc, oracle_mod, use_diff):
    """photo 2048 x 2048 (> 2^20 block symbols: the shipping build's parallel pass): the oracle's
    stream decodes to the input; damaged copies report the oracle's status and bytes"""
    torch = gpu
    W = H = 2048
    m = oracle_mod.synth("photo", 3, W, H)
    if use_diff:
        m = np.frombuffer(oracle_mod.diff(m), dtype=np.uint8)
    st, stream, _ = oracle_mod.adapt(m, W, H)
    assert st == 0
    hdr, x = _adaptive_parts(oracle_mod, stream)
    assert len(x) >= 1 << 20
    rng = np.random.default_rng(11)
    cases = [x] + _damaged(rng, x)
    datas = [B.container(oracle_mod, hdr + y) for y in cases]
    wants = [oracle_mod.decompress(d) for d in datas]
    assert wants[0] == (0, m.tobytes())  # (the container's flags carry no diff bit)
    dst, dec, _ = decompress_adapt_batch(hc, torch, datas, [W * H] * len(datas))
    for k, ((wst, want), gst, got) in enumerate(zip(wants, dst, dec)):
        assert gst == wst, (k, gst, wst)
        if wst == 0:
            assert got == want, k


def test_par_bounds_real_threshold_constant_runs(gpu, hc, oracle_mod):
    """a forged stream of 8 x 8 blocks that are all [b, b, b, 61] (the no-reset machine never
    rejoins a reset one inside these runs): > 2^20 block symbols, valid and damaged"""
    torch = gpu
    W = H = 4096
    b = 8
    nb = (W // b) * (H // b)
    hdr = list(W.to_bytes(8, "big") + H.to_bytes(8, "big") + b.to_bytes(8, "big")) + [0xA5] * (nb // 8)
    x = [5, 5, 5, 61] * nb
    rng = np.random.default_rng(5)
    cases = [x] + _damaged(rng, x)
    datas = [B.container(oracle_mod, hdr + y) for y in cases]
    wants = [oracle_mod.decompress(d) for d in datas]
    assert wants[0][0] == 0
    dst, dec, _ = decompress_adapt_batch(hc, torch, datas, [W * H] * len(datas))
    for k, ((wst, want), gst, got) in enumerate(zip(wants, dst, dec)):
        assert gst == wst, (k, gst, wst)
        if wst == 0:
            assert got == want, k


@pytest.mark.parametrize("skew", [1, 4099, 777777])
def test_par_bounds_wrong_entries_repaired(gpu, hc, oracle_mod, skew):
    """every odd chunk of the parallel pass walks from a wrong entry (hc_debug_set_par_skew): its
    walk writes block starts under wrong block numbers, racing with the neighbouring chunks' walks.
    par_fix must re-run those chunks and rewrite the entries they touched: the decoded bytes and
    statuses still equal the oracle's (valid and damaged streams, threshold 0 and real sizes)."""
    torch = gpu
    hc.use_debug_build(True)
    hc.debug_set_par_min(0)
    hc.debug_set_par_skew(skew)
    try:
        datas, wants, sizes = [], [], []
        rng = np.random.default_rng(skew)
        for k, (W, H, use_diff) in enumerate([(2048, 2048, True), (512, 512, False), (512, 512, True),
                                              (1024, 768, True)]):
            m = oracle_mod.synth("photo", k, W, H)
            if use_diff:
                m = np.frombuffer(oracle_mod.diff(m), dtype=np.uint8)
            st, stream, _ = oracle_mod.adapt(m, W, H)
            assert st == 0
            hdr, x = _adaptive_parts(oracle_mod, stream)
            for y in [x] + _damaged(rng, x)[:2]:
                d = B.container(oracle_mod, hdr + y)
                datas.append(d)
                wants.append(oracle_mod.decompress(d))
                sizes.append(W * H)
        dst, dec, _ = decompress_adapt_batch(hc, torch, datas, sizes)
        for k, ((wst, want), gst, got) in enumerate(zip(wants, dst, dec)):
            assert gst == wst, (k, gst, wst)
            if wst == 0:
                assert got == want, k
    finally:
        hc.debug_set_par_skew(0)
        hc.debug_set_par_min(1 << 20)
        hc.use_debug_build(False)


def test_par_bounds_no_block_symbols(gpu, hc, oracle_mod, par_everywhere):
    """blocks announced, no block symbol at all (count == header): the reference exits with 14
    (transform.cpp:170-174). With the parallel pass's threshold at 0 such a stream still goes
    through the serial pass: dec_header_kernel marks a stream parallel only when it holds block
    symbols, and the serial pass is what reports 14 here."""
    torch = gpu
    W = H = 64
    b = 8
    nb = (W // b) * (H // b)
    hdr = list(W.to_bytes(8, "big") + H.to_bytes(8, "big") + b.to_bytes(8, "big")) + [0xFF] * (nb // 8)
    datas = [B.container(oracle_mod, hdr), B.container(oracle_mod, hdr + [7])]
    wants = [oracle_mod.decompress(d) for d in datas]
    assert wants[0][0] == 14
    dst, dec, _ = decompress_adapt_batch(hc, torch, datas, [W * H] * len(datas))
    assert dst == [w[0] for w in wants]
