"""The adaptive-RLE kernels' arithmetic (tests/adapt_cost_model.py) against the oracle: the
bit-string segment monoid gives |applyRLE(x)| exactly (long runs, 258-chunk edges, random),
the per-tile evaluation (Eh / Ev words, substituted first bits) gives every block's h / v
cost at every block size, the tile pieces give the blocks larger than a tile, the emit rule
reproduces applyRLE byte for byte, and choosing + assembling reproduces applyAdaptRLE
(transform.cpp:294-328) — so the kernels built on these pieces are pinned before they run."""
import random

import pytest

import adapt_cost_model as M


def _runs(rng, n, maxrun, alphabet):
    out = []
    while len(out) < n:
        out += [rng.randrange(alphabet)] * rng.randint(1, maxrun)
    return out[:n]


def test_rle_length_edges(oracle_mod):
    for L in list(range(1, 40)) + list(range(250, 270)) + list(range(510, 530)) + [774, 775, 776, 1032, 2000]:
        for tail in ([], [7], [7, 7], [7, 9, 9, 9]):
            seq = [5] * L + tail
            assert M.rle_len_via_bits(seq) == len(oracle_mod.rle(bytes(seq))), (L, tail)
            assert M.emit_lanes(seq) == list(oracle_mod.rle(bytes(seq))), (L, tail)


def test_rle_length_random(oracle_mod):
    rng = random.Random(7)
    for k in range(400):
        n = rng.randint(1, 3000)
        seq = _runs(rng, n, rng.choice([1, 3, 6, 300, 900]), rng.choice([2, 3, 256]))
        want = oracle_mod.rle(bytes(seq))
        assert M.rle_len_via_bits(seq) == len(want)
        assert M.emit_lanes(seq) == list(want)


def test_seg_join_any_split():
    rng = random.Random(3)
    for _ in range(200):
        bits = [0] + [int(rng.random() < 0.8) for _ in range(rng.randint(0, 700))]
        whole = M.fold_bits(bits)
        cut = rng.randint(0, len(bits))
        a, b = M.fold_bits(bits[:cut]), M.fold_bits(bits[cut:])
        j = M.seg_join(a, b)
        assert (j.n, j.lead, j.tail, j.mid) == (whole.n, whole.lead, whole.tail, whole.mid)


def test_counted_cost(oracle_mod):
    """the kernel's pattern-count cost for whole-tile blocks (B = 8..64: 64..4096 elements)
    equals |applyRLE| whenever it applies (no all-ones word); runs of 1..300 elements"""
    rng = random.Random(5)
    used = 0
    for k in range(600):
        n = rng.choice([64, 256, 1024, 4096])
        seq = _runs(rng, n, rng.choice([1, 3, 6, 40, 70, 300]), rng.choice([2, 3, 256]))
        got = M.counted_cost(M.bits_of(seq))
        if got is not None:
            used += 1
            assert got == len(oracle_mod.rle(bytes(seq))), (k, n)
        else:
            assert n > 258
    assert used > 300


def _matrix(kind, W, H, seed):
    rng = random.Random(seed)
    if kind == "flat":
        return [3] * (W * H)
    if kind == "bands":  # long horizontal runs, equal rows: long runs in both scan orders
        return [(y // 37) & 1 for y in range(H) for x in range(W)]
    if kind == "runs":
        return _runs(rng, W * H, 40, 3)
    return [rng.randrange(4) for _ in range(W * H)]


@pytest.mark.parametrize("kind", ["flat", "bands", "runs", "noise4"])
@pytest.mark.parametrize("W,H", [(136, 72), (64, 200), (8, 8), (129, 9), (200, 131)])
def test_tiled_block_costs(oracle_mod, kind, W, H):
    m = _matrix(kind, W, H, W * 31 + H)
    for use_diff in (False, True):
        D = M.diffed(m, use_diff)
        B = 8
        while B <= min(W, H, 128):
            got = M.block_costs_tiled(m, W, H, B, use_diff)
            for i, (hc, vc) in enumerate(got):
                x0, y0, sx, sy = M.block_geo(W, H, B, i)
                assert hc == len(oracle_mod.rle(bytes(M.scan(D, W, x0, y0, sx, sy, True)))), (B, i)
                assert vc == len(oracle_mod.rle(bytes(M.scan(D, W, x0, y0, sx, sy, False)))), (B, i)
            B *= 2


@pytest.mark.parametrize("kind", ["flat", "bands", "runs"])
def test_big_block_costs_from_tile_pieces(oracle_mod, kind):
    W, H = 300, 270
    m = _matrix(kind, W, H, 11)
    for use_diff in (False, True):
        D = M.diffed(m, use_diff)
        hp, vp = M.tile_pieces(m, W, H, use_diff)
        B = 256
        nb = (-(-W // B)) * (-(-H // B))
        for i in range(nb):
            x0, y0, sx, sy = M.block_geo(W, H, B, i)
            hc, vc = M.big_block_cost(hp, vp, W, H, B, i)
            assert hc == len(oracle_mod.rle(bytes(M.scan(D, W, x0, y0, sx, sy, True))))
            assert vc == len(oracle_mod.rle(bytes(M.scan(D, W, x0, y0, sx, sy, False))))


def test_choose_and_assemble_is_apply_adapt(oracle_mod):
    """argmin over block sizes (first minimum of header + data), per-block h/v choice (tie ->
    h), header, block RLEs in order == the oracle's applyAdaptRLE output"""
    for kind, W, H in (("runs", 136, 72), ("bands", 64, 200), ("noise4", 40, 24)):
        m = _matrix(kind, W, H, 5)
        best = None
        B, steps = 8, 0
        while steps <= 7 and B <= W and B <= H:
            costs = M.block_costs_tiled(m, W, H, B)
            nb = len(costs)
            total = 24 + (nb + 7) // 8 + sum(min(h, v) for h, v in costs)
            if best is None or total < best[0]:
                best = (total, B, costs)
            B *= 2
            steps += 1
        total, B, costs = best
        dirs = [int(h <= v) for h, v in costs]
        out = bytearray(W.to_bytes(8, "big") + H.to_bytes(8, "big") + B.to_bytes(8, "big"))
        for k in range(0, len(dirs), 8):
            byte = 0
            for j in range(8):
                byte = byte << 1 | (dirs[k + j] if k + j < len(dirs) else 0)
            out.append(byte)
        for i, d in enumerate(dirs):
            x0, y0, sx, sy = M.block_geo(W, H, B, i)
            out += bytes(M.emit_lanes(M.scan(m, W, x0, y0, sx, sy, bool(d))))
        assert len(out) == total
        st, want, wb = oracle_mod.adapt(bytes(m), W, H)
        assert st == 0 and wb == B and bytes(out) == want
