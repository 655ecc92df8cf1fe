"""CPU checks of the parallel block-boundary model (tests/bounds_par_model.py, the algorithm of
hc_adapt.hip's bounds_par kernels) against the serial process of revertAdaptRLE
(transform.cpp:330-361 / 162-187), itself checked against the oracle's adaptive revert."""
import random

import numpy as np
import pytest

import bounds_par_model as M


def block_symbols(rng, want, p_rep=0.6, alpha=4):
    """MNP-5 symbols decoding to exactly `want` bytes (literals, runs, counts incl. zero)"""
    out, got, prev, rep = [], 0, 0, 0
    while got < want:
        if rep == 3:
            c = rng.randint(0, min(want - got, 255))
            out.append(c)
            got += c
            rep = 0
            continue
        v = prev if rng.random() < p_rep else rng.randrange(alpha)
        out.append(v)
        got += 1
        rep = rep + 1 if (v == prev and rep) else 1
        prev = v
    return out


def synthetic(rng, W, H, B, **kw):
    x = []
    for want in M.block_wants(W, H, B):
        x += block_symbols(rng, want, **kw)
    return x


def check(x, W, H, B, chunk):
    st, starts = M.serial(x, W, H, B)
    pst, pstarts, stats = M.parallel(x, W, H, B, chunk=chunk)
    assert pst == st
    if st == 0:
        assert pstarts == starts
    return stats


def test_serial_model_matches_oracle(oracle_mod):
    """the model's serial process reports the oracle's status on valid and damaged streams"""
    rng = random.Random(3)
    for case in range(12):
        W, H, B = rng.randint(8, 70), rng.randint(8, 70), rng.choice([8, 16, 32])
        x = synthetic(rng, W, H, B)
        if case % 3 == 1:
            x = x[:-rng.randint(1, 4)]
        elif case % 3 == 2:
            x = x + [1, 2]
        nb = -(-W // B) * -(-H // B)
        hdr = W.to_bytes(8, "big") + H.to_bytes(8, "big") + B.to_bytes(8, "big") + bytes(-(-nb // 8))
        want_st, _ = oracle_mod.unadapt(hdr + bytes(x))
        assert M.serial(x, W, H, B)[0] == want_st


@pytest.mark.parametrize("chunk", [17, 64, 300])
def test_parallel_equals_serial_random_blocks(chunk):
    """small blocks (B = 8: 64-byte blocks of a few symbols, windows reaching past block ends),
    counts (zero counts included) and their corruptions"""
    rng = random.Random(chunk)
    for case in range(40):
        W, H, B = rng.randint(8, 60), rng.randint(8, 60), rng.choice([8, 8, 16, 32])
        x = synthetic(rng, W, H, B, p_rep=rng.choice([0.3, 0.6, 0.9]), alpha=rng.choice([2, 4, 64]))
        kind = case % 4
        if kind == 1:
            x = x[: max(0, len(x) - rng.randint(1, 6))]
        elif kind == 2:
            x = x + [rng.randrange(4) for _ in range(rng.randint(1, 4))]
        elif kind == 3 and x:
            j = rng.randrange(len(x))
            x[j] = (x[j] + rng.randint(1, 255)) & 255
        check(x, W, H, B, chunk)


def test_parallel_constant_runs():
    """long constant runs ([b, b, b, count] repeated): the no-reset machine never rejoins a
    reset one inside them (windows longer than the Z cap)"""
    for B in (8, 16):
        W = H = 48
        x = []
        for want in M.block_wants(W, H, B):
            while want > 0:
                c = min(want - 3, 255) if want > 3 else 0
                if want >= 3:
                    x += [5, 5, 5, c]
                    want -= 3 + c
                else:
                    x += [5] * want
                    want = 0
        check(x, W, H, B, 50)


def test_parallel_on_encoder_output(oracle_mod):
    """adaptive streams the encoder writes (photo 256x256, with and without the diff model):
    few block starts need the scanner's correction and no chunk is re-run"""
    for use_diff in (False, True):
        m = oracle_mod.synth("photo", 1, 256, 256)
        if use_diff:
            m = np.frombuffer(oracle_mod.diff(m), dtype=np.uint8)
        st = np.frombuffer(oracle_mod.adapt(m, 256, 256)[1], dtype=np.uint8)
        W, H, B = (int.from_bytes(st[8 * i:8 * i + 8].tobytes(), "big") for i in range(3))
        nb = -(-W // B) * -(-H // B)
        x = st[24 + -(-nb // 8):].tolist()
        stats = check(x, W, H, B, 2048)
        assert stats["reruns"] == 0
