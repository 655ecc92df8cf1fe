"""GPU parity of the encoder's two ways of finding a symbol's code and root path.

Cache mode keeps the root paths of recently coded symbols (hc_fgk.hip Fgk::pc_*); table mode
keeps the decoder's level tables plus each position's code (pcode[]) and checks every lookup
against the tables (hc_fgk.hip code_all_tab); the small-alphabet kernel is cache mode with exact
15-symbol steps while a stream has seen <= 16 symbols (tests/test_gpu_small.py).
hc_debug_set_enc_tab forces one mode for every stream, and each must produce the reference's bytes: its digests, edge vectors, deep / skewed trees (vs the oracle)
and the adaptive symbol streams; by default (mode 0) enc_mode_kernel picks per stream. Reference: huffman.cpp:136-155 (code of a symbol),
huffman.cpp:95-128 (update), transform.cpp:363-384 (applyHuffman).
"""
import hashlib

import pytest

from gpu_batch import compress_adapt_batch, compress_batch, decompress_adapt_batch, decompress_batch
from test_gpu_parity import _deep_and_skewed

pytestmark = pytest.mark.gpu


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(params=[2, 1, 3, 0], ids=["tables", "cache", "small", "auto"])
def enc_mode(request, gpu, hc):
    hc.use_debug_build(True)  # the hook exists in the debug build only
    hc.debug_set_enc_tab(request.param)
    yield request.param
    hc.debug_set_enc_tab(0)
    hc.use_debug_build(False)


def test_enc_mode_digests(gpu, hc, oracle_mod, digests, enc_mode):
    torch = gpu
    names = [f"{kind}_{k}" for kind in ("photo", "grad", "noise") for k in range(4)]
    raws = [oracle_mod.synth(n.split("_")[0], int(n.split("_")[1])).tobytes() for n in names]
    for mode in ("c", "cm"):
        st, encs, _ = compress_batch(hc, torch, raws, mode == "cm")
        assert st == [0] * len(raws)
        for n, e in zip(names, encs):
            want = digests["synthetic"][n][mode]
            assert (len(e), sha(e)) == (want["len"], want["sha256"]), (n, mode)
        st, back, _ = decompress_batch(hc, torch, encs, [len(r) for r in raws])
        assert st == [0] * len(raws) and back == raws


def test_enc_mode_vectors_and_trees(gpu, hc, oracle_mod, vectors, enc_mode):
    torch = gpu
    for mode in ("c", "cm"):
        vs = [v for v in vectors["compress"] if v["mode"] == mode]
        st, encs, _ = compress_batch(hc, torch, [bytes.fromhex(v["input"]) for v in vs], mode == "cm")
        assert st == [0] * len(vs)
        for v, e in zip(vs, encs):
            assert e.hex() == v["output"], (v["name"], mode)
    raws = _deep_and_skewed()
    for use_diff in (False, True):
        st, encs, _ = compress_batch(hc, torch, raws, use_diff)
        assert st == [0] * len(raws)
        for i, (r, e) in enumerate(zip(raws, encs)):
            ost, want = oracle_mod.compress(r, use_diff, False, 512)
            assert ost == 0 and e == want, (i, use_diff)


def test_enc_mode_adaptive(gpu, hc, oracle_mod, digests, enc_mode):
    torch = gpu
    raws = [oracle_mod.synth("photo", k).tobytes() for k in range(3)]
    for mode in ("ca", "cma"):
        st, encs, _ = compress_adapt_batch(hc, torch, raws, [512] * 3, mode == "cma")
        assert st == [0] * 3
        for k, e in enumerate(encs):
            w = digests["synthetic"][f"photo_{k}"][mode]
            assert (len(e), sha(e)) == (w["len"], w["sha256"]), (k, mode)
        st, back, _ = decompress_adapt_batch(hc, torch, encs, [len(r) for r in raws])
        assert st == [0] * 3 and back == raws
