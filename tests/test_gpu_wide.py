"""GPU parity of the wide FGK variants on non-adaptive streams.

The kernels switch to the 32-bit weight layout ("wide") once a stream can exceed 2^22 - 2
symbols: the encoder for raw inputs over ~3.1 MB (n + n/3 + 2 > 2^22 - 2), the decoder for
counts over 2^22 - 2 (hc_fgk.hip: encode_kernel / decode_kernel). These inputs are the only
ones that reach encode_kernel<1, SRC_RAW | SRC_RAW_DIFF> and decode_kernel<1, DST_RAW>;
their outputs are compared with the reference binary's digests (tests/golden/digests.json
"wide", made by tests/golden/make_golden_wide.py from oracle/_ref/huffman-codec-O2):

  2048x2048 photo / grad / noise  wide encode (noise -c: also a wide decode, 4194307 symbols)
  4096x4096 photo                 wide encode and decode (-c: 12.9 M symbols)

Reference: transform.cpp:363-406 (applyHuffman / revertHuffman), huffman.hpp:26 (u64 freq).
"""
import hashlib

import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

NARROW_MAX = (1 << 22) - 2


def sha(b):
    return hashlib.sha256(b).hexdigest()


def _synth(torch, hc, kind, side):
    buf = torch.empty(side * side, dtype=torch.uint8, device="cuda")
    hc.synth_batch(kind, 0, 1, side, side, buf, 0)
    torch.cuda.synchronize()
    return buf


def test_wide_goldens_cover_both_variants(digests):
    w = digests["wide"]
    assert w["photo_0_4096"]["c"]["count"] > NARROW_MAX      # wide decode
    assert w["noise_0_2048"]["c"]["count"] > NARROW_MAX      # wide decode at 4 MiB
    assert w["photo_0_2048"]["cm"]["count"] <= NARROW_MAX    # wide encode, narrow decode
    for name, e in w.items():
        n = e["side"] ** 2
        assert n + n // 3 + 2 > NARROW_MAX, name              # every one a wide encode


@pytest.mark.parametrize("mode", ["c", "cm"])
def test_wide_single_api_4096(gpu, hc, digests, mode):
    """hc_compress / hc_decompress (single-buffer API) on the 4096x4096 photo"""
    torch = gpu
    e = digests["wide"]["photo_0_4096"]
    raw = _synth(torch, hc, "photo", 4096).cpu().numpy().tobytes()
    assert sha(raw) == e["raw_sha256"]
    st, out = hc.compress(raw, mode == "cm", False, 512)
    assert st == 0
    assert (len(out), sha(out)) == (e[mode]["len"], e[mode]["sha256"])
    st, back = hc.decompress(out)
    assert st == 0 and back == raw


@pytest.mark.parametrize("mode", ["c", "cm"])
def test_wide_batch_api(gpu, hc, digests, mode):
    """hc_compress_batch / hc_decompress_batch on one batch holding every wide case"""
    torch = gpu
    names = sorted(digests["wide"])
    raws = []
    for name in names:
        kind, _, side = name.split("_")
        raws.append(_synth(torch, hc, kind, int(side)))
    n = len(raws)
    lens = [r.numel() for r in raws]
    offs, o = [], 0
    for L in lens:
        offs.append(o)
        o += (L + 255) // 256 * 256
    din = torch.zeros(o, dtype=torch.uint8, device="cuda")
    for r, off in zip(raws, offs):
        din[off:off + r.numel()] = r
    caps = [hc.compress_bound(L) for L in lens]
    eoffs, o = [], 0
    for c in caps:
        eoffs.append(o)
        o += (c + 255) // 256 * 256
    enc = torch.zeros(o, dtype=torch.uint8, device="cuda")
    t = lambda v: torch.tensor(v, dtype=torch.int64, device="cuda")
    elens = torch.zeros(n, dtype=torch.int64, device="cuda")
    est = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    hc.compress_batch(din, t(offs), t(lens), enc, t(eoffs), t(caps), elens, est, use_diff=(mode == "cm"))
    torch.cuda.synchronize()
    assert est.cpu().tolist() == [0] * n
    eh = enc.cpu().numpy()
    el = elens.cpu().tolist()
    for name, off, L in zip(names, eoffs, el):
        want = digests["wide"][name][mode]
        out = eh[off:off + L].tobytes()
        assert (len(out), sha(out)) == (want["len"], want["sha256"]), name
    back = torch.zeros_like(din)
    blens = torch.zeros(n, dtype=torch.int64, device="cuda")
    bst = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    hc.decompress_batch(enc, t(eoffs), elens, back, t(offs), t(lens), blens, bst)
    torch.cuda.synchronize()
    assert bst.cpu().tolist() == [0] * n
    assert blens.cpu().tolist() == lens
    for name, r, off in zip(names, raws, offs):
        assert torch.equal(back[off:off + r.numel()], r), name
