"""Streams beyond the 32-bit buffer offsets (the reference counts in u64,
huffman.hpp:26, main.cpp:93-94).

The FGK kernels reach a stream's input and output through buffer windows that slide forward
once the offset inside them passes g_window (1 GiB). Two checks:
  * with the window shrunk to 4 KiB (hc_debug_set_window), ordinary streams cross hundreds of
    window edges in every direction (encoder input, encoder output words, decoder input bits,
    decoder output bytes, narrow and wide trees): byte-identical to the oracle / the reference's
    digests, round trips exact;
  * one real 4.5 GiB stream (-c): input and raw output far past 2^32 bytes, byte-identical to the
    oracle, round trip exact.
"""
import hashlib

import numpy as np
import pytest

from gpu_batch import compress_batch, decompress_batch

pytestmark = pytest.mark.gpu


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture
def small_window(gpu, hc):
    hc.use_debug_build(True)  # the hook exists in the debug build only
    hc.debug_set_window(4096)
    yield
    hc.debug_set_window(1 << 30)
    hc.use_debug_build(False)


def test_small_window_batch_vs_oracle(gpu, hc, oracle_mod, small_window):
    torch = gpu
    raws = [oracle_mod.synth(k, i, w, h).tobytes() for i, (k, w, h) in
            enumerate([("photo", 512, 512), ("noise", 512, 1024), ("grad", 700, 300), ("photo", 33, 17)])]
    raws.append(bytes(300000))
    for use_diff in (False, True):
        st, enc, _ = compress_batch(hc, torch, raws, use_diff)
        assert st == [0] * len(raws)
        for r, e in zip(raws, enc):
            want_st, want = oracle_mod.compress(r, use_diff, False, 512)
            assert want_st == 0 and e == want
        dst, dec, _ = decompress_batch(hc, torch, enc, [len(r) for r in raws])
        assert dst == [0] * len(raws) and dec == raws


@pytest.mark.timeout(600)
def test_small_window_wide_digests(gpu, hc, digests, small_window):
    """the 4096x4096 photo through the wide trees (12.9 M symbols), windows of 4 KiB"""
    torch = gpu
    e = digests["wide"]["photo_0_4096"]
    buf = torch.empty(4096 * 4096, dtype=torch.uint8, device="cuda")
    hc.synth_batch("photo", 0, 1, 4096, 4096, buf, 0)
    raw = buf.cpu().numpy().tobytes()
    st, out = hc.compress(raw, False, False, 512)
    assert st == 0 and (len(out), sha(out)) == (e["c"]["len"], e["c"]["sha256"])
    st, back = hc.decompress(out)
    assert st == 0 and back == raw


@pytest.mark.timeout(900)
def test_stream_past_4_gib(gpu, hc, oracle_mod):
    """4.5 GiB of mostly constant bytes (-c): a few changes at both sides of 2^31 and 2^32"""
    torch = gpu
    n = (9 << 29)  # 4.5 GiB
    raw = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    for p in ((1 << 31) - 3, (1 << 31) + 1, (1 << 32) - 2, (1 << 32), (1 << 32) + 5, n - 1):
        raw[p] = (p * 31) & 255
    cap = 64 << 20
    enc = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    i64 = dict(dtype=torch.int64, device="cuda")
    z = torch.zeros(1, **i64)
    elen = torch.zeros(1, **i64)
    est = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    hc.compress_batch(raw, z, torch.tensor([n], **i64), enc, z, torch.tensor([cap], **i64), elen, est)
    torch.cuda.synchronize()
    assert est.item() == 0
    got = enc[:elen.item()].cpu().numpy().tobytes()
    host = raw.cpu().numpy()
    want_st, want = oracle_mod.compress(host, False, False, 512)
    assert want_st == 0 and got == want
    del host
    back = torch.zeros_like(raw)
    blen = torch.zeros(1, **i64)
    bst = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    hc.decompress_batch(enc, z, elen, back, z, torch.tensor([n], **i64), blen, bst)
    torch.cuda.synchronize()
    assert bst.item() == 0 and blen.item() == n
    assert torch.equal(back, raw)
