"""The batched hot paths (tests/fgk_batch_model.py; hc_fgk.hip code_all_batch, Dec::decode_batch)
code every symbol as the one-symbol loop does and leave the same tree, on the photo / grad / noise
streams with and without the diff model and on the deep / skewed alphabets of the GPU tests."""
import numpy as np
import pytest

from fgk_batch_model import encode


def _streams(oracle_mod):
    out = []
    for kind in ("photo", "grad", "noise"):
        raw = oracle_mod.synth(kind, 3, 160, 120).tobytes()
        out.append(oracle_mod.rle(oracle_mod.diff(raw)))
        out.append(oracle_mod.rle(raw))
    rng = np.random.default_rng(5)
    zipf = 1.0 / np.arange(1, 257) ** 1.1
    out.append(rng.choice(256, 20000, p=zipf / zipf.sum()).astype(np.uint8).tobytes())
    sym, a, b = [], 1, 1
    for s in range(16):
        sym += [(s * 37) & 255] * a
        a, b = b, a + b
    out.append(rng.permutation(np.array(sym, dtype=np.uint8)).tobytes())
    out.append(b"\x00\xff" * 3000)
    return out


@pytest.mark.parametrize("misses,exact,retry,small", [(False, False, False, False), (False, False, True, False),
                                                      (False, True, False, False), (True, True, False, False),
                                                      (False, False, False, True)])
def test_batched_equals_one_symbol_loop(oracle_mod, misses, exact, retry, small):
    total = {"batches": 0, "alone": 0, "n": 0}
    for k, syms in enumerate(_streams(oracle_mod) + _small_streams()):
        syms = list(syms)
        c1, t1, _ = encode(syms, batched=False)
        c2, t2, st = encode(syms, batched=True, misses=misses, exact=exact, retry=retry, small=small)
        assert c1 == c2, k
        assert t1.w == t2.w and t1.body == t2.body and t1.up == t2.up, k
        total["batches"] += st["batches"]
        total["alone"] += st["alone"]
        total["n"] += len(syms)
    assert total["batches"] < total["n"]


@pytest.mark.parametrize("retry", [False, True])
def test_decoder_batches_equal_one_symbol_loop(oracle_mod, retry):
    """Dec::decode_batch's tentative commit (every batch symbol counted before each level test),
    with and without the retest, leaves the tree of the one-symbol loop and fails no level the
    exact counts pass"""
    from fgk_batch_model import decode
    total = {"batches": 0, "alone": 0, "n": 0}
    for k, syms in enumerate(_streams(oracle_mod)):
        syms = list(syms)
        t1, _ = decode(syms, batched=False)
        t2, st = decode(syms, batched=True, retry=retry)
        assert t1.w == t2.w and t1.body == t2.body and t1.up == t2.up, k
        total["batches"] += st["batches"]
        total["alone"] += st["alone"]
        total["n"] += len(syms)
    assert total["batches"] < total["n"]


def _small_streams():
    """streams that stay within 16 symbols (the encoder's small-alphabet steps) or cross the limit:
    skewed few-symbol mixes, exact ties, a ramp of growing alphabets, deep paths (Fibonacci)"""
    rng = np.random.default_rng(11)
    out = []
    for n_sym in (2, 3, 5, 9, 16, 17, 24):
        p = rng.random(n_sym) ** 3
        out.append(rng.choice(rng.permutation(256)[:n_sym], 6000, p=p / p.sum()).astype(np.uint8).tobytes())
    out.append(bytes([1, 2, 3, 4] * 1500))  # four symbols in lockstep: every update ties
    out.append(bytes(sum(([s] * (3 + s % 5) for s in range(40)), [])) * 20)  # the alphabet grows past 16
    sym, a, b = [], 1, 1
    for s_ in range(12):  # a deep tree within 16 symbols
        sym += [s_ * 19 & 255] * a
        a, b = b, a + b
    out.append(rng.permutation(np.array(sym, dtype=np.uint8)).tobytes())
    return out


def test_small_alphabet_steps_on_grad(oracle_mod):
    """the encoder's small-alphabet steps (fgk_batch_model.small_len: exact counts, 15 symbols of
    depth <= 4 per step) on grad -c -m: 319 steps and 13 symbols alone per 512x512 stream, where
    the tentative 7-symbol batches take 1034 and 523"""
    raw = oracle_mod.synth("grad", 0, 512, 512).tobytes()
    syms = list(oracle_mod.rle(oracle_mod.diff(raw)))
    c1, t1, _ = encode(syms, batched=False)
    c2, t2, st = encode(syms, batched=True, small=True)
    assert c1 == c2 and t1.w == t2.w and t1.body == t2.body
    assert st == {"batches": 0, "alone": 13, "small": 319}


def test_retry_on_grad(oracle_mod):
    """the retest takes grad's false failures (an earlier batch symbol through the next position)
    out of the batches: per 512x512 grad -c -m stream 1034 batches and 523 symbols alone with the
    tentative test alone, 671 and 15 with the retest (the exact counts: 670 and 14)"""
    raw = oracle_mod.synth("grad", 0, 512, 512).tobytes()
    syms = list(oracle_mod.rle(oracle_mod.diff(raw)))
    c1, t1, _ = encode(syms, batched=False)
    c2, t2, st = encode(syms, batched=True, retry=True)
    assert c1 == c2 and t1.w == t2.w
    assert st == {"batches": 671, "alone": 15}
    _, st0 = encode(syms, batched=True)[1:]
    assert st0 == {"batches": 1034, "alone": 523}
