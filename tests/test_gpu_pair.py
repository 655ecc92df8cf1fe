"""GPU parity of the two-streams-per-wavefront decoder (hc_fgk.hip decode2_kernel / decode_pair:
streams A and B on lanes 0-31 / 32-63 of one wavefront, in lockstep while both have symbols, then
the longer one alone), enabled through the debug build's hc_debug_set_dec_pair. It is not the
shipping decoder (one stream per wavefront measured faster on C5), but it stays
bit-exact: the parity tests' batches decode through it, against the oracle and the reference's
digests, including odd batch sizes (a wavefront with one stream), partners of very different
lengths (the pair ends inside a block), and malformed partners (a stream that stops early)."""
import numpy as np
import pytest

import test_gpu_parity as P
from gpu_batch import compress_batch, decompress_batch

pytestmark = pytest.mark.gpu


@pytest.fixture
def pair(gpu, hc):
    hc.use_debug_build(True)
    hc.debug_set_dec_pair(True)
    yield
    hc.debug_set_dec_pair(False)
    hc.use_debug_build(False)


@pytest.mark.parametrize("mode", ["c", "cm"])
def test_pair_synthetic_512_digests(gpu, hc, oracle_mod, digests, mode, pair):
    P.test_batch_synthetic_512_digests(gpu, hc, oracle_mod, digests, mode)


def test_pair_mixed_sizes(gpu, hc, oracle_mod, pair):
    P.test_batch_vs_oracle_mixed_sizes(gpu, hc, oracle_mod)


def test_pair_deep_and_skewed(gpu, hc, oracle_mod, pair):
    P.test_batch_deep_and_skewed(gpu, hc, oracle_mod)


def test_pair_edge_vectors(gpu, hc, vectors, pair):
    P.test_batch_edge_vectors(gpu, hc, vectors)


def test_pair_decode_malformed(gpu, hc, vectors, pair):
    P.test_batch_decode_malformed(gpu, hc, vectors)


def test_pair_partners(gpu, hc, oracle_mod, vectors, pair):
    """every pairing of a long photo stream with: a shorter one ending mid-block, one ending on a
    block edge, an empty one, a malformed one; in both orders; an odd batch size"""
    torch = gpu
    long = oracle_mod.synth("photo", 5, 300, 200).tobytes()
    others = [oracle_mod.synth("noise", 1, 50, 37).tobytes(), b"\x07" * 600, b"",
              oracle_mod.synth("grad", 2, 64, 64).tobytes()]
    raws = []
    for o in others:
        raws += [long, o, o, long]
    raws.append(long)  # odd count: the last wavefront holds one stream
    for use_diff in (False, True):
        st, encs, _ = compress_batch(hc, torch, raws, use_diff)
        assert st == [0] * len(raws)
        bad = [v for v in vectors["decompress"] if not v["name"].startswith("a_") and v["rc"]][:3]
        encs2, wants = [], []
        for k, e in enumerate(encs):
            encs2.append(e)
            wants.append((0, raws[k]))
        for v in bad:
            encs2 += [bytes.fromhex(v["input"]), encs[0]]
            wants += [(v["rc"], None), (0, raws[0])]
        dst, back, _ = decompress_batch(hc, torch, encs2, [max(len(r), 1) for r in raws] + [1 << 20] * (len(encs2) - len(raws)))
        for k, ((wst, want), s, b) in enumerate(zip(wants, dst, back)):
            assert s == wst, (k, s, wst)
            if want is not None:
                assert b == want, k
