"""GPU parity of the adaptive decoder's block-boundary search (hc_adapt.hip: bounds_kernel,
transform.cpp:330-361 running revertRLEBlock transform.cpp:162-187 block by block).

Adaptive symbol streams are built directly (header + per-block MNP-5 data), wrapped in the
outer container with the oracle's FGK coder, and decoded by the GPU and by the oracle; status
and bytes must agree. Blocks are small and ragged (W, H not multiples of B) so that many blocks
close inside one 256-symbol step, counts land on block ends (including zero counts), and the
corrupted variants hit exit codes 13 (a count overshoots its block), 14 (the stream ends inside
a block) and 15 (symbols left after the last block).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def block_symbols(rng, want):
    """MNP-5 symbols decoding to exactly `want` bytes (literals, runs with counts, zero counts)."""
    out, got, prev, rep = [], 0, 0, 0
    while got < want:
        left = want - got
        if rep == 3:  # the machine expects a count
            c = int(rng.integers(0, min(left, 255) + 1))
            out.append(c)
            got += c
            rep = 0
            continue
        v = prev if rng.random() < 0.6 else int(rng.integers(0, 4))
        out.append(v)
        got += 1
        rep = rep + 1 if (v == prev and rep) else 1
        prev = v
    return out


def container(oracle_mod, stream):
    payload, _ = oracle_mod.fgk_encode(bytes(stream))
    return len(stream).to_bytes(8, "little") + b"\x40" + payload


def adaptive_stream(rng, w, h, b):
    nb = -(-w // b) * -(-h // b)
    hdr = list(w.to_bytes(8, "big") + h.to_bytes(8, "big") + b.to_bytes(8, "big"))
    hdr += list(rng.integers(0, 256, size=-(-nb // 8), dtype=np.uint8).tobytes())
    body = []
    per_row = -(-w // b)
    for i in range(nb):
        x0, y0 = (i % per_row) * b, (i // per_row) * b
        body += block_symbols(rng, min(b, w - x0) * min(b, h - y0))
    return hdr, body


def test_bounds_valid_and_corrupted_vs_oracle(gpu, hc, oracle_mod):
    rng = np.random.default_rng(2026)
    seen = set()
    for case in range(60):
        w, h = int(rng.integers(8, 90)), int(rng.integers(8, 90))
        b = int(rng.choice([8, 16, 32]))
        hdr, body = adaptive_stream(rng, w, h, b)
        kind = case % 5
        if kind == 1:  # drop symbols at the end: the last block starves (14) or is cut (13)
            body = body[: max(0, len(body) - int(rng.integers(1, 6)))]
        elif kind == 2:  # extra symbols after the last block (15)
            body = body + [int(v) for v in rng.integers(0, 4, size=int(rng.integers(1, 4)))]
        elif kind == 3:  # one symbol changed somewhere: desynchronises every later block
            k = int(rng.integers(0, len(body)))
            body[k] = (body[k] + int(rng.integers(1, 256))) & 255
        elif kind == 4:  # random symbols of a plausible length
            body = [int(v) for v in rng.choice([0, 0, 1, 1, 1, 2, 3, 200], size=len(body))]
        data = container(oracle_mod, hdr + body)
        want_st, want = oracle_mod.decompress(data)
        st, got = hc.decompress(data)
        assert st == want_st, (case, w, h, b, kind)
        if st == 0:
            assert got == want, (case, w, h, b)
        seen.add(st)
    assert {0, 13, 14, 15} <= seen, seen


def test_bounds_many_blocks_per_step(gpu, hc, oracle_mod):
    """B = 8 over a 200 x 120 matrix: 375 blocks of ~40 symbols, several close per step"""
    rng = np.random.default_rng(7)
    hdr, body = adaptive_stream(rng, 200, 120, 8)
    data = container(oracle_mod, hdr + body)
    want_st, want = oracle_mod.decompress(data)
    st, got = hc.decompress(data)
    assert want_st == 0 and st == 0 and got == want


def test_bounds_other_block_sizes_vs_oracle(gpu, hc, oracle_mod):
    """block sizes a forged header may carry besides 8..128: B >= 256 (one start entry per
    block) and sizes that are not powers of two (K-block groups, K > 1 for small blocks), ragged
    matrices with several block rows and groups; valid, starved and overlong streams"""
    rng = np.random.default_rng(99)
    seen = set()
    cases = [(300, 270, 256), (530, 260, 256), (520, 300, 512), (100, 90, 3), (77, 41, 5), (130, 70, 12),
             (200, 150, 24), (333, 121, 40), (250, 260, 100), (610, 300, 300), (64, 64, 7), (90, 200, 9)]
    for case, (w, h, b) in enumerate(cases):
        hdr, body = adaptive_stream(rng, w, h, b)
        kind = case % 3
        if kind == 1:
            body = body[: max(0, len(body) - int(rng.integers(1, 6)))]
        elif kind == 2:
            body = body + [int(v) for v in rng.integers(0, 4, size=int(rng.integers(1, 4)))]
        data = container(oracle_mod, hdr + body)
        want_st, want = oracle_mod.decompress(data)
        st, got = hc.decompress(data)
        assert st == want_st, (case, w, h, b, kind)
        if st == 0:
            assert got == want, (case, w, h, b)
        seen.add(st)
    assert 0 in seen and len(seen) >= 2, seen


def test_bounds_narrow_forged_matrices_vs_oracle(gpu, hc, oracle_mod):
    """forged headers the encoder never writes: matrices 1..3 wide (or high) with B = 8 / 16,
    whose tile block rows outnumber the group-start entries a W, H >= 8 stream needs (the decoder
    then takes K-block groups instead). Decoded through the batched API with the exact output
    capacity (W * H) and through the single-buffer API; status and bytes as the oracle's
    (headers.cpp:65-105 accepts any W, H; transform.cpp:330-361)."""
    from gpu_batch import decompress_adapt_batch
    torch = gpu
    rng = np.random.default_rng(31)
    streams, sizes, wants = [], [], []
    for (w, h, b) in [(1, 3000, 8), (2, 2000, 8), (3, 1200, 8), (1, 4000, 16), (2, 900, 16), (3000, 1, 8),
                      (3, 3, 8), (1, 1, 8)]:
        hdr, body = adaptive_stream(rng, w, h, b)
        data = container(oracle_mod, hdr + body)
        want_st, want = oracle_mod.decompress(data)
        assert want_st == 0, (w, h, b)
        st, got = hc.decompress(data)
        assert st == 0 and got == want, (w, h, b)
        streams.append(data)
        sizes.append(w * h)
        wants.append(want)
    dst, dec, _ = decompress_adapt_batch(hc, torch, streams, sizes)
    assert dst == [0] * len(streams)
    assert dec == wants
