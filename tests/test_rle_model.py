"""The encoder's lane-parallel MNP-5 pre-pass (hc_fgk.hip: rle_chunk), as a numpy model
(tests/rle_chunk_model.py), equals the reference's serial FSM (oracle, transform.cpp:241-279)
on run structures around every 258-byte cut and 256-byte chunk boundary."""
import numpy as np
import pytest

from rle_chunk_model import rle_chunked


def test_chunked_rle_equals_serial(oracle_mod):
    rng = np.random.default_rng(0)
    lens = [1, 2, 3, 4, 255, 256, 257, 258, 259, 260, 515, 516, 517, 773, 774, 775]
    for t in range(600):
        data = b"".join(bytes([int(rng.integers(0, 3))]) * int(rng.choice(lens + [int(rng.integers(1, 900))]))
                        for _ in range(int(rng.integers(1, 25))))
        if t % 5 == 0:
            data = data[: int(rng.integers(0, len(data) + 1))]
        for diff in (False, True):
            want = oracle_mod.rle(oracle_mod.diff(data) if diff else data)
            assert rle_chunked(data, diff) == want, (t, diff)
    for k in range(6):
        raw = oracle_mod.synth(("photo", "grad", "noise")[k % 3], k, 64, 64).tobytes()
        for diff in (False, True):
            assert rle_chunked(raw, diff) == oracle_mod.rle(oracle_mod.diff(raw) if diff else raw)


# ---- decoder side: lane-parallel RLE + diff revert (tests/revert_block_model.py)
import random as _random

import revert_block_model as _rb


def test_revert_block_model_streams(oracle_mod):
    for kind in ("photo", "grad", "noise"):
        raw = oracle_mod.synth(kind, 2, 128, 96).tobytes()
        for diff in (True, False):
            sym = oracle_mod.rle(oracle_mod.diff(raw) if diff else raw)
            assert _rb.revert_blocked(sym, diff) == raw, (kind, diff)


def test_revert_block_model_random(oracle_mod):
    rng = _random.Random(11)
    for t in range(120):
        n = rng.randrange(0, 1100)
        alpha = rng.choice([2, 3, 5, 256])
        sym = bytes(rng.randrange(alpha) for _ in range(n))
        for diff in (True, False):
            want = oracle_mod.unrle(sym)
            if diff:
                want = oracle_mod.undiff(want)
            assert _rb.revert_blocked(sym, diff) == want, (t, diff)



def test_pure_chunk_fast_path(oracle_mod):
    """the encoder's fast path for a chunk of 256 copies of the carried byte (rle_chunk_model.
    pure_chunk) inside the chunked pass equals the reference's FSM, for every run counter R the
    carry can hold when such a chunk starts (0..257) and both diff settings"""
    for c in (0, 1, 200):
        for R in range(258):
            for diff in (False, True):
                # stream: filler chunk(s), then a run of c whose counter reaches R at a chunk
                # edge, then 1-3 pure chunks, then a different byte and a short tail
                body = bytes([c]) * (R if R else 258)
                head = bytes([(c + 7) & 255]) * ((-len(body)) % 256 or 256)
                raw = head + body + bytes([c]) * (256 * (1 + R % 3)) + bytes([(c + 9) & 255, c, c])
                if diff:  # a stream whose diff is raw (prefix sums)
                    raw = np.cumsum(np.frombuffer(raw, dtype=np.uint8), dtype=np.uint64).astype(np.uint8).tobytes()
                want = oracle_mod.rle(oracle_mod.diff(raw) if diff else raw)
                assert rle_chunked(raw, diff, fast=True) == want, (c, R, diff)


def _run_heavy(rng, n):
    """a stream of runs (lengths around the 258-byte cut and the 1 KB block) with sparse and dense
    stretches, as raw bytes whose diff (or themselves) carry those runs"""
    lens = [1, 2, 3, 4, 255, 256, 257, 258, 259, 260, 300, 515, 516, 517, 773, 1023, 1024, 1025, 2100]
    parts, tot = [], 0
    while tot < n:
        if rng.random() < 0.15:  # a dense stretch
            k = int(rng.integers(16, 700))
            parts.append(rng.integers(0, 256, k).astype(np.uint8).tobytes())
        else:
            k = int(rng.choice(lens))
            parts.append(bytes([int(rng.integers(0, 4))]) * k)
        tot += k
    return b"".join(parts)[:n]


@pytest.mark.parametrize("block", [2048, 1024])
def test_blocked_rle_equals_serial(oracle_mod, block, monkeypatch):
    """the encoder's sparse blocks (rle_chunk_model.rle_blocked, hc_fgk.hip rle_block; 2 KB as
    shipped, 1 KB the HC_SPARSE_KB=1 build) inside the chunk loop equal the reference's FSM
    (transform.cpp:241-279): run-heavy streams with dense stretches, every carried counter phase,
    both diff settings, and the grad photos"""
    import rle_chunk_model
    from rle_chunk_model import rle_blocked
    monkeypatch.setattr(rle_chunk_model, "kBlock", block)
    rng = np.random.default_rng(5)
    for t in range(160):
        data = _run_heavy(rng, int(rng.integers(1, 24000)))
        for diff in (False, True):
            raw = data
            if diff:  # a stream whose diff is `data`
                raw = np.cumsum(np.frombuffer(data, dtype=np.uint8), dtype=np.uint64).astype(np.uint8).tobytes()
            want = oracle_mod.rle(oracle_mod.diff(raw) if diff else raw)
            assert rle_blocked(raw, diff) == want, (t, diff)
    for k in range(3):
        raw = oracle_mod.synth("grad", k, 512, 64).tobytes()
        for diff in (False, True):
            assert rle_blocked(raw, diff) == oracle_mod.rle(oracle_mod.diff(raw) if diff else raw)


def test_block_edge_vectors_cover_every_carried_phase(oracle_mod):
    """the 2 KB block-edge vectors of tests/test_gpu_sparse.py (_edge_streams): in the model of the
    kernel's loop every one of them codes the blocks at 256 + 2048 and 256 + 4096 sparse, the run
    counter carried into the block at 256 + 4096 takes all 258 phases over the set, and the output
    equals the reference's FSM in both diff settings"""
    from rle_chunk_model import rle_blocked
    from test_gpu_sparse import _edge_streams
    phases = set()
    for i, raw in enumerate(_edge_streams()):
        for diff in (False, True):
            if diff:
                raw = np.cumsum(np.frombuffer(raw, dtype=np.uint8), dtype=np.uint64).astype(np.uint8).tobytes()
            blocks = []
            assert rle_blocked(raw, diff, blocks) == oracle_mod.rle(oracle_mod.diff(raw) if diff else raw), (i, diff)
            at = dict(blocks)
            assert 256 + 2048 in at and 256 + 4096 in at, (i, diff, blocks[:4])
            phases.add(at[256 + 4096])
    assert phases == set(range(258))
