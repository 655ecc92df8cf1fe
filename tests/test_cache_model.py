"""CPU checks of the FGK kernels' path cache and level tables (tests/fgk_cache_model.py): every
cached path and every table lookup equals the plain slot-form tree's answer, on symbol streams
of the synthetic kinds, the -m transform and hand-made deep / flat / swap-heavy sequences."""
import random

import pytest

import fgk_cache_model as M


def _streams(oracle_mod):
    out = []
    for kind in ("photo", "grad", "noise"):
        raw = oracle_mod.synth(kind, 3, 128, 96).tobytes()
        out.append((kind + " -m", oracle_mod.rle(oracle_mod.diff(raw))))
        out.append((kind, oracle_mod.rle(raw)))
    return out


def test_cache_model_synthetic(oracle_mod):
    for name, sym in _streams(oracle_mod):
        r = M.run(list(sym))
        assert r["n"] == len(sym), name


@pytest.mark.parametrize("seed", range(4))
def test_cache_model_random(seed):
    rng = random.Random(seed)
    # skewed alphabet: a few hot symbols (cache hits) among many cold ones (swaps, splits)
    alphabet = list(range(256))
    weights = [1.0 / (1 + i) ** 1.2 for i in range(256)]
    rng.shuffle(alphabet)
    sym = rng.choices(alphabet, weights, k=6000)
    M.run(sym)


def test_cache_model_fibonacci_deep():
    # Fibonacci-like counts build codes far deeper than the tables' 8 levels
    sym = []
    a, b = 1, 1
    for s in range(20):
        sym += [s] * a
        a, b = b, a + b
    random.Random(7).shuffle(sym)
    M.run(sym[:8000])


def test_cache_model_edges():
    M.run([])
    M.run([5])
    M.run([5] * 300)
    M.run(list(range(256)) * 3)


def _lockstep(symbols):
    """The kernels' update (lane-parallel test, walk with chase-back) leaves exactly the tree
    of the plain slot-form update after every symbol."""
    ref, ker = M.Tree(), M.Tree()
    for s in symbols:
        for t in (ref, ker):
            if t.where[s] == 0:
                t.split(s)
        x = ref.where[s]
        assert ker.where[s] == x
        ref.update(x)
        M.kernel_update(ker, x, ker.path(x) + [M.ROOT])
        assert ref.w == ker.w and ref.body == ker.body and ref.up == ker.up


def test_kernel_update_streams(oracle_mod):
    for name, sym in _streams(oracle_mod):
        _lockstep(list(sym))


@pytest.mark.parametrize("seed", range(3))
def test_kernel_update_random(seed):
    rng = random.Random(100 + seed)
    alphabet = list(range(256))
    weights = [1.0 / (1 + i) ** rng.choice([0.5, 1.2, 2.0]) for i in range(256)]
    rng.shuffle(alphabet)
    _lockstep(rng.choices(alphabet, weights, k=5000))
