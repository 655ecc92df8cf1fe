"""The encoder's lane-parallel MNP-5 pre-pass (hc_fgk.hip: rle_chunk), as a numpy model
(tests/rle_chunk_model.py), equals the reference's serial FSM (oracle, transform.cpp:241-279)
on run structures around every 258-byte cut and 256-byte chunk boundary."""
import numpy as np

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
