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
