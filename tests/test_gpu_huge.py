"""Streams of 2^32 - 1 symbols and more: the "huge" FGK tree layout (64-bit weights).

The reference counts in u64 (HuffNode::freq, huffman.hpp:26; the u64 header count,
headers.cpp:107-125, main.cpp:93-94), so a stream may hold any number of FGK symbols. The
kernels pick the tree layout from the stream's (worst-case) symbol count: narrow (22-bit
weights packed with the parent), wide (32-bit weights) or huge (64-bit weights, hc_fgk.hip
tree_kind). Coding one real stream past 2^32 symbols takes minutes per direction (one serial
wavefront), so these tests force every stream onto the wide or the huge layout
(hc_debug_set_min_tree) and check the kernels bit for bit on ordinary inputs: the reference's
digests, its edge and malformed-stream vectors, the deep / skewed trees against the oracle, and
both adaptive entry points. test_huge_real_stream_encode / _decode (opt-in: HC_HUGE_REAL=enc /
dec, ~10 minutes each on one wavefront) code one stream of 2^32 + 2^20 symbols against the
oracle; their logs are kept under profiles/.
"""
import hashlib
import os
import time

import numpy as np
import pytest

from gpu_batch import compress_adapt_batch, compress_batch, decompress_adapt_batch, decompress_batch
from test_gpu_parity import _deep_and_skewed

pytestmark = pytest.mark.gpu


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(params=[1, 2], ids=["wide", "huge"])
def tree(request, gpu, hc):
    hc.use_debug_build(True)  # the hook exists in the debug build only
    hc.debug_set_min_tree(request.param)
    yield request.param
    hc.debug_set_min_tree(0)
    hc.use_debug_build(False)


def test_forced_tree_digests(gpu, hc, oracle_mod, digests, tree):
    """512x512 synthetic streams k = 0..3 of every kind, -c and -c -m: the reference's digests"""
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


def test_forced_tree_vectors(gpu, hc, vectors, tree):
    """the reference's edge vectors (RLE cut points, last-byte rule, empty, all 256, deep) and
    its malformed streams (status codes 8 / 9, accepted forgeries byte for byte)"""
    torch = gpu
    for mode in ("c", "cm"):
        vs = [v for v in vectors["compress"] if v["mode"] == mode]
        raws = [bytes.fromhex(v["input"]) for v in vs]
        st, encs, _ = compress_batch(hc, torch, raws, mode == "cm")
        assert st == [0] * len(vs)
        for v, e in zip(vs, encs):
            assert e.hex() == v["output"], (v["name"], mode)
        st, back, _ = decompress_batch(hc, torch, encs, [len(r) for r in raws])
        assert back == raws
    vs = [v for v in vectors["decompress"] if not v["name"].startswith("a_")]
    st, outs, _ = decompress_batch(hc, torch, [bytes.fromhex(v["input"]) for v in vs], [1 << 20] * len(vs))
    for v, s, o in zip(vs, st, outs):
        assert s == v["rc"], v["name"]
        if s == 0:
            assert o.hex() == v["output"], v["name"]


def test_forced_tree_deep_and_skewed(gpu, hc, oracle_mod, tree):
    """Fibonacci-deep codes, Zipf, flat and alternating alphabets: every swap / walk / descent path"""
    torch = gpu
    raws = _deep_and_skewed()
    for use_diff in (False, True):
        st, encs, _ = compress_batch(hc, torch, raws, use_diff)
        assert st == [0] * len(raws)
        for i, (r, e) in enumerate(zip(raws, encs)):
            ost, want = oracle_mod.compress(r, use_diff, False, 512)
            assert ost == 0 and e == want, (i, use_diff)
        st, back, _ = decompress_batch(hc, torch, encs, [len(r) for r in raws])
        assert st == [0] * len(raws) and back == raws


def test_forced_tree_adaptive(gpu, hc, oracle_mod, digests, vectors, tree):
    """-a / -a -m through the symbol-stream kernels (SRC_SYMBOLS / DST_SYMBOLS): the single-buffer
    API and the batched adaptive API against the reference's digests, and the adaptive error
    vectors (status codes 10 / 11 / 13 / 14 / 15)"""
    torch = gpu
    raws = [oracle_mod.synth("photo", k).tobytes() for k in range(3)]
    for mode in ("ca", "cma"):
        want = digests["synthetic"]["photo_0"][mode]
        st, out = hc.compress(raws[0], mode == "cma", True, 512)
        assert st == 0 and (len(out), sha(out)) == (want["len"], want["sha256"]), mode
        st, back = hc.decompress(out)
        assert st == 0 and back == raws[0]
        st, encs, _ = compress_adapt_batch(hc, torch, raws, [512] * 3, mode == "cma")
        assert st == [0] * 3
        for k, e in enumerate(encs):
            w = digests["synthetic"][f"photo_{k}"][mode]
            assert (len(e), sha(e)) == (w["len"], w["sha256"]), (k, mode)
        st, back, _ = decompress_adapt_batch(hc, torch, encs, [len(r) for r in raws])
        assert st == [0] * 3 and back == raws
    vs = [v for v in vectors["decompress"] if v["name"].startswith("a_")]
    st, _, _ = decompress_adapt_batch(hc, torch, [bytes.fromhex(v["input"]) for v in vs], [1 << 20] * len(vs))
    assert st == [v["rc"] for v in vs]


def test_header_count_past_u32(gpu, hc, oracle_mod):
    """A header announcing 2^32 + 7 symbols is decoded as the reference does (no device limit):
    with a short payload status 9 (transform.cpp:394-398), like the oracle"""
    torch = gpu
    _, enc = oracle_mod.compress(oracle_mod.synth("photo", 0, 64, 64).tobytes(), True, False, 512)
    forged = ((1 << 32) + 7).to_bytes(8, "little") + enc[8:]
    ost, _ = oracle_mod.decompress(forged)
    st, _, _ = decompress_batch(hc, torch, [forged], [1 << 16])
    assert st == [ost] == [9]


def _huge_input(torch):
    n = (1 << 32) + (1 << 20)
    pat = torch.tensor([1, 1, 2, 1, 1, 3, 1, 1, 2], dtype=torch.uint8, device="cuda")
    return n, pat.repeat(n // pat.numel() + 1)[:n].contiguous()


@pytest.mark.timeout(1100)
@pytest.mark.skipif(os.environ.get("HC_HUGE_REAL") != "enc", reason="opt-in: ~10 minutes on one wavefront")
def test_huge_real_stream_encode(gpu, hc, oracle_mod):
    """one stream of 2^32 + 2^20 FGK symbols (-c on a 4 GiB input without runs of 3, so every
    byte is a symbol): the GPU encoding is byte for byte the oracle's (u64 weights)"""
    torch = gpu
    n, raw = _huge_input(torch)
    cap = n // 2
    enc = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    i64 = dict(dtype=torch.int64, device="cuda")
    z = torch.zeros(1, **i64)
    elen = torch.zeros(1, **i64)
    est = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    t0 = time.time()
    hc.compress_batch(raw, z, torch.tensor([n], **i64), enc, z, torch.tensor([cap], **i64), elen, est)
    torch.cuda.synchronize()
    print(f"gpu encode {time.time() - t0:.1f} s", flush=True)
    assert est.item() == 0
    got = enc[:elen.item()].cpu().numpy()
    assert int.from_bytes(got[:8].tobytes(), "little") == n  # every byte a symbol
    host = raw.cpu().numpy()
    del raw
    t0 = time.time()
    want_st, want = oracle_mod.compress(host, False, False, 512)
    print(f"oracle encode {time.time() - t0:.1f} s", flush=True)
    assert want_st == 0 and len(want) == len(got) and np.array_equal(np.frombuffer(want, np.uint8), got)


@pytest.mark.timeout(1100)
@pytest.mark.skipif(os.environ.get("HC_HUGE_REAL") != "dec", reason="opt-in: ~12 minutes on one wavefront")
def test_huge_real_stream_decode(gpu, hc, oracle_mod):
    """the oracle's encoding of the same 2^32 + 2^20-symbol stream decoded on the GPU (huge tree
    layout picked from the header count): exactly the input"""
    torch = gpu
    n, raw = _huge_input(torch)
    t0 = time.time()
    want_st, want = oracle_mod.compress(raw.cpu().numpy(), False, False, 512)
    print(f"oracle encode {time.time() - t0:.1f} s", flush=True)
    assert want_st == 0 and int.from_bytes(want[:8], "little") == n
    enc = torch.from_numpy(np.frombuffer(want, np.uint8).copy()).cuda()
    del want
    i64 = dict(dtype=torch.int64, device="cuda")
    z = torch.zeros(1, **i64)
    back = torch.zeros_like(raw)
    blen = torch.zeros(1, **i64)
    bst = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    t0 = time.time()
    hc.decompress_batch(enc, z, torch.tensor([enc.numel()], **i64), back, z, torch.tensor([n], **i64), blen, bst)
    torch.cuda.synchronize()
    print(f"gpu decode {time.time() - t0:.1f} s", flush=True)
    assert bst.item() == 0 and blen.item() == n
    assert torch.equal(back, raw)
