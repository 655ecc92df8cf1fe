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


@pytest.mark.parametrize("misses,exact", [(False, False), (False, True), (True, True)])
def test_batched_equals_one_symbol_loop(oracle_mod, misses, exact):
    total = {"batches": 0, "alone": 0, "n": 0}
    for k, syms in enumerate(_streams(oracle_mod)):
        syms = list(syms)
        c1, t1, _ = encode(syms, batched=False)
        c2, t2, st = encode(syms, batched=True, misses=misses, exact=exact)
        assert c1 == c2, k
        assert t1.w == t2.w and t1.body == t2.body and t1.up == t2.up, k
        total["batches"] += st["batches"]
        total["alone"] += st["alone"]
        total["n"] += len(syms)
    assert total["batches"] < total["n"]


def test_decoder_batches_equal_one_symbol_loop(oracle_mod):
    """Dec::decode_batch's tentative commit (every batch symbol counted before each level test)
    leaves the tree of the one-symbol loop and fails no level the exact counts pass"""
    from fgk_batch_model import decode
    total = {"batches": 0, "alone": 0, "n": 0}
    for k, syms in enumerate(_streams(oracle_mod)):
        syms = list(syms)
        t1, _ = decode(syms, batched=False)
        t2, st = decode(syms, batched=True)
        assert t1.w == t2.w and t1.body == t2.body and t1.up == t2.up, k
        total["batches"] += st["batches"]
        total["alone"] += st["alone"]
        total["n"] += len(syms)
    assert total["batches"] < total["n"]
