"""GPU parity: the HIP path (through the C ABI) against the oracle and the reference's goldens.

Bit-exact is the bar everywhere (integer / byte work). Sizes where the pointer-tree oracle
finishes in seconds are compared with the oracle directly; the 512x512 and 4096x4096 cases
are compared with SHA-256 digests the reference binary produced (tests/golden/digests.json).
"""
import hashlib
import os

import numpy as np
import pytest

from gpu_batch import compress_batch, decompress_batch

pytestmark = pytest.mark.gpu

MODES = {"c": (False, False), "cm": (True, False), "ca": (False, True), "cma": (True, True)}
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_device_synth_matches_oracle(gpu, hc, oracle_mod, digests):
    torch = gpu
    for kind in ("photo", "grad", "noise"):
        buf = torch.empty(4 * 262144, dtype=torch.uint8, device="cuda")
        hc.synth_batch(kind, 0, 4, 512, 512, buf, 262144)
        torch.cuda.synchronize()
        h = buf.cpu().numpy()
        for k in range(4):
            assert sha(h[k * 262144:(k + 1) * 262144].tobytes()) == digests["synthetic"][f"{kind}_{k}"]["raw_sha256"]
    buf = torch.empty(517 * 300 + 3, dtype=torch.uint8, device="cuda")
    hc.synth_batch("photo", 7, 1, 517, 300, buf, 0)
    torch.cuda.synchronize()
    assert buf[:517 * 300].cpu().numpy().tobytes() == oracle_mod.synth("photo", 7, 517, 300).tobytes()


@pytest.mark.parametrize("mode", ["c", "cm"])
def test_batch_synthetic_512_digests(gpu, hc, oracle_mod, digests, mode):
    """12 reference outputs at 512x512 (photo / grad / noise, k = 0..3), bit for bit."""
    torch = gpu
    names = sorted(digests["synthetic"])
    raws = [oracle_mod.synth(n.split("_")[0], int(n.split("_")[1])).tobytes() for n in names]
    st, encs, _ = compress_batch(hc, torch, raws, use_diff=(mode == "cm"))
    assert st == [0] * len(raws)
    for n, e in zip(names, encs):
        want = digests["synthetic"][n][mode]
        assert (len(e), sha(e)) == (want["len"], want["sha256"]), n
    st, back, _ = decompress_batch(hc, torch, encs, [len(r) for r in raws])
    assert st == [0] * len(raws)
    assert back == raws


@pytest.mark.parametrize("mode", ["c", "cm"])
def test_batch_synthetic_digests_full_launch(gpu, hc, oracle_mod, digests, mode):
    """the same 12 reference outputs inside a batch of 264 streams (the same input in a launch
    that fills more than one wave per CU, repeated streams in one launch)"""
    torch = gpu
    names = sorted(digests["synthetic"])
    base = [oracle_mod.synth(n.split("_")[0], int(n.split("_")[1])).tobytes() for n in names]
    raws = base * 22
    st, encs, _ = compress_batch(hc, torch, raws, use_diff=(mode == "cm"))
    assert st == [0] * len(raws)
    for k, e in enumerate(encs):
        want = digests["synthetic"][names[k % len(names)]][mode]
        assert (len(e), sha(e)) == (want["len"], want["sha256"]), k
    st, back, _ = decompress_batch(hc, torch, encs, [len(r) for r in raws])
    assert st == [0] * len(raws) and back == raws


def test_batch_vs_oracle_mixed_sizes(gpu, hc, oracle_mod):
    """ragged batch: lengths not multiples of 4, tiny and empty streams, both modes"""
    torch = gpu
    rng = np.random.default_rng(11)
    raws = [b"", b"\x01", b"\x00\x00\x00", b"\x05" * 258, b"\x05" * 259 + b"\x06"]
    for k in range(40):
        w, h = int(rng.integers(1, 160)), int(rng.integers(1, 90))
        kind = ("photo", "grad", "noise")[k % 3]
        raws.append(oracle_mod.synth(kind, 100 + k, w, h).tobytes()[: w * h - int(rng.integers(0, 3))])
    for use_diff in (False, True):
        st, encs, _ = compress_batch(hc, torch, raws, use_diff)
        assert st == [0] * len(raws)
        for r, e in zip(raws, encs):
            ost, want = oracle_mod.compress(r, use_diff, False, 512)
            assert ost == 0 and e == want, len(r)
        st, back, _ = decompress_batch(hc, torch, encs, [len(r) for r in raws])
        assert st == [0] * len(raws) and back == raws


def _deep_and_skewed():
    """Symbol streams that stress the tree rather than the transforms: Fibonacci counts (codes
    deeper than the decoder's 8 table levels and the encoder's cached paths, up to the
    reference's ~24-bit worst case), a Zipf alphabet (hot cached symbols among many cold ones:
    swaps that drop cache entries), all 256 symbols round robin (a flat tree, no repeats for
    the first 256 symbols), two symbols alternating (swap every symbol), sorted runs."""
    rng = np.random.default_rng(23)
    out = []
    for n_fib in (12, 20, 24):
        sym, a, b = [], 1, 1
        for s in range(n_fib):
            sym += [(s * 37) & 255] * a
            a, b = b, a + b
        sym = np.array(sym, dtype=np.uint8)
        out.append(sym.tobytes())                   # ascending counts, unshuffled
        out.append(rng.permutation(sym).tobytes())  # the same counts shuffled
    zipf = 1.0 / np.arange(1, 257) ** 1.1
    out.append(rng.choice(256, 150000, p=zipf / zipf.sum()).astype(np.uint8).tobytes())
    out.append(bytes(range(256)) * 300)
    out.append(b"\x00\xff" * 40000)
    out.append(np.repeat(np.arange(256, dtype=np.uint8), 200).tobytes())
    return out


def test_batch_deep_and_skewed(gpu, hc, oracle_mod):
    torch = gpu
    raws = _deep_and_skewed()
    for use_diff in (False, True):
        st, encs, _ = compress_batch(hc, torch, raws, use_diff)
        assert st == [0] * len(raws)
        for i, (r, e) in enumerate(zip(raws, encs)):
            ost, want = oracle_mod.compress(r, use_diff, False, 512)
            assert ost == 0 and e == want, (i, len(r), use_diff)
        st, back, _ = decompress_batch(hc, torch, encs, [len(r) for r in raws])
        assert st == [0] * len(raws) and back == raws


def test_batch_deep_and_skewed_full_launch(gpu, hc, oracle_mod):
    """the deep / skewed streams repeated in a launch of 260 streams"""
    torch = gpu
    base = _deep_and_skewed()
    raws = (base * (257 // len(base) + 1))[:260]
    for use_diff in (False, True):
        wants = [oracle_mod.compress(r, use_diff, False, 512) for r in base]
        st, encs, _ = compress_batch(hc, torch, raws, use_diff)
        assert st == [0] * len(raws)
        for i, e in enumerate(encs):
            assert wants[i % len(base)][0] == 0 and e == wants[i % len(base)][1], (i, use_diff)
        st, back, _ = decompress_batch(hc, torch, encs, [len(r) for r in raws])
        assert st == [0] * len(raws) and back == raws


def test_batch_flat_and_skewed_segments(gpu, hc, oracle_mod):
    """Streams whose alphabet turns flat and skewed again, segment by segment (noise, photo,
    grad): the decoder switches its batches off and on per 256-symbol block by their yield (and
    probes every 8th block), the encoder's batches stop at every uncached symbol; every stream
    equals the oracle and round-trips"""
    torch = gpu
    raws = []
    for k in range(6):
        parts = []
        for j, kind in enumerate(("noise", "photo", "noise", "grad", "photo", "noise")[k % 3:]):
            parts.append(oracle_mod.synth(kind, 40 + 7 * k + j, 256, 96 + 32 * (j % 3)).tobytes())
        raws.append(b"".join(parts))
    for use_diff in (False, True):
        st, encs, _ = compress_batch(hc, torch, raws, use_diff)
        assert st == [0] * len(raws)
        for i, (r, e) in enumerate(zip(raws, encs)):
            ost, want = oracle_mod.compress(r, use_diff, False, 512)
            assert ost == 0 and e == want, (i, len(r), use_diff)
        st, back, _ = decompress_batch(hc, torch, encs, [len(r) for r in raws])
        assert st == [0] * len(raws) and back == raws


def test_batch_edge_vectors(gpu, hc, vectors):
    torch = gpu
    for mode in ("c", "cm"):
        vs = [v for v in vectors["compress"] if v["mode"] == mode]
        raws = [bytes.fromhex(v["input"]) for v in vs]
        st, encs, _ = compress_batch(hc, torch, raws, use_diff=(mode == "cm"))
        assert st == [0] * len(vs)
        for v, e in zip(vs, encs):
            assert e.hex() == v["output"], (v["name"], mode)
        st, back, _ = decompress_batch(hc, torch, encs, [len(r) for r in raws])
        assert back == raws


def test_batch_decode_malformed(gpu, hc, vectors):
    torch = gpu
    vs = [v for v in vectors["decompress"] if not v["name"].startswith("a_")]
    encs = [bytes.fromhex(v["input"]) for v in vs]
    st, outs, _ = decompress_batch(hc, torch, encs, [1 << 20] * len(encs))
    for v, s, o in zip(vs, st, outs):
        assert s == v["rc"], v["name"]
        if s == 0:
            assert o.hex() == v["output"], v["name"]


def test_batch_capacity_reporting(gpu, hc, oracle_mod):
    torch = gpu
    raw = oracle_mod.synth("photo", 2, 64, 64).tobytes()
    _, want = oracle_mod.compress(raw, True, False, 512)
    st, encs, lens = compress_batch(hc, torch, [raw], True, cap_fn=lambda n: 100)
    assert st == [hc.HC_ERR_CAPACITY] and lens == [len(want)]
    st, encs, lens = compress_batch(hc, torch, [raw], True, cap_fn=lambda n: len(want))
    assert st == [0] and encs == [want]
    st, outs, lens = decompress_batch(hc, torch, [want], [len(raw) - 1])
    assert st == [hc.HC_ERR_CAPACITY] and lens == [len(raw)]


@pytest.mark.parametrize("mode", list(MODES))
def test_single_api_vs_oracle(gpu, hc, oracle_mod, mode):
    d, a = MODES[mode]
    for kind, k, w, h in (("photo", 9, 96, 80), ("grad", 2, 64, 64), ("noise", 1, 40, 33),
                          ("photo", 4, 517, 40)):
        raw = oracle_mod.synth(kind, k, w, h).tobytes()
        st, out = hc.compress(raw, d, a, w)
        ost, want = oracle_mod.compress(raw, d, a, w)
        assert st == ost == 0 and out == want, (kind, mode)
        st, back = hc.decompress(out)
        assert st == 0 and back == raw


def test_single_api_adaptive_vectors(gpu, hc, vectors):
    for v in vectors["adaptive"]:
        d, a = MODES[v["mode"]]
        st, out = hc.compress(bytes.fromhex(v["input"]), d, a, v["width"])
        assert st == v["rc"], v["name"]
        assert out.hex() == v["output"], (v["name"], v["mode"])
        if st == 0:
            st, back = hc.decompress(out)
            assert st == 0 and back.hex() == v["input"]


def test_single_api_decode_malformed(gpu, hc, vectors):
    for v in vectors["decompress"]:
        st, out = hc.decompress(bytes.fromhex(v["input"]))
        assert st == v["rc"], v["name"]
        if st == 0:
            assert out.hex() == v["output"], v["name"]


def test_corpus_huf_decode_and_reencode(gpu, hc, digests):
    """the reference's own outputs for sample images: decode, check the raw digest, re-encode"""
    for fn in sorted(os.listdir(os.path.join(GOLDEN, "corpus"))):
        name, mode, _ = fn.split(".")
        huf = open(os.path.join(GOLDEN, "corpus", fn), "rb").read()
        st, raw = hc.decompress(huf)
        assert st == 0 and sha(raw) == digests["corpus"][name]["raw_sha256"], fn
        d, a = MODES[mode]
        st, again = hc.compress(raw, d, a, 512)
        assert st == 0 and again == huf, fn


def test_synthetic_512_adaptive_digests(gpu, hc, oracle_mod, digests):
    for name in ("photo_0", "grad_1", "noise_2"):
        kind, k = name.split("_")
        raw = oracle_mod.synth(kind, int(k)).tobytes()
        for mode in ("ca", "cma"):
            d, a = MODES[mode]
            st, out = hc.compress(raw, d, a, 512)
            want = digests["synthetic"][name][mode]
            assert st == 0 and (len(out), sha(out)) == (want["len"], want["sha256"]), (name, mode)
            st, back = hc.decompress(out)
            assert st == 0 and back == raw


def test_adaptive_4096_digest(gpu, hc, digests):
    """config C4: -c -a -w 4096 on one 4096x4096 photo matrix (wide-tree FGK, 11.7M symbols)"""
    torch = gpu
    buf = torch.empty(4096 * 4096, dtype=torch.uint8, device="cuda")
    hc.synth_batch("photo", 0, 1, 4096, 4096, buf, 0)
    torch.cuda.synchronize()
    raw = buf.cpu().numpy().tobytes()
    e = digests["synthetic_4096"]["photo_0"]
    assert sha(raw) == e["raw_sha256"]
    for mode in ("ca", "cma"):
        d, a = MODES[mode]
        st, out = hc.compress(raw, d, a, 4096)
        assert st == 0 and (len(out), sha(out)) == (e[mode]["len"], e[mode]["sha256"]), mode
        st, back = hc.decompress(out)
        assert st == 0 and back == raw


@pytest.mark.parametrize("n,use_diff", [(1024, True), (4096, False)], ids=["1024-cm", "C3-4096-c"])
def test_roundtrip_property_full_batch(gpu, hc, digests, n, use_diff):
    """size-independent properties at full batch shapes (1024 photo streams -c -m; config C3:
    4096 streams -c, where the batch vote puts the encoder in table mode): decode(encode(x)) == x,
    the encoded sizes are deterministic across two launches, and streams 0..3 (photo k = 0..3)
    match the reference's digests"""
    torch = gpu
    N = 262144
    raw = torch.empty(n * N, dtype=torch.uint8, device="cuda")
    hc.synth_batch("photo", 0, n, 512, 512, raw, N)
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * N
    lens = torch.full((n,), N, dtype=torch.int64, device="cuda")
    cap = 2 * N
    enc = torch.empty(n * cap, dtype=torch.uint8, device="cuda")
    eoffs = torch.arange(n, dtype=torch.int64, device="cuda") * cap
    ecaps = torch.full((n,), cap, dtype=torch.int64, device="cuda")
    elens = torch.zeros(n, dtype=torch.int64, device="cuda")
    st = torch.zeros(n, dtype=torch.int32, device="cuda")
    hc.compress_batch(raw, offs, lens, enc, eoffs, ecaps, elens, st, use_diff=use_diff)
    elens2 = torch.zeros_like(elens)
    hc.compress_batch(raw, offs, lens, enc, eoffs, ecaps, elens2, st, use_diff=use_diff)
    back = torch.empty_like(raw)
    blens = torch.zeros_like(lens)
    st2 = torch.zeros_like(st)
    hc.decompress_batch(enc, eoffs, elens, back, offs, lens, blens, st2)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0 and int(st2.abs().sum()) == 0
    assert torch.equal(elens, elens2)
    assert torch.equal(blens, lens)
    assert torch.equal(back, raw)
    mode = "cm" if use_diff else "c"
    for k in range(4):
        e = enc[k * cap:k * cap + int(elens[k])].cpu().numpy().tobytes()
        want = digests["synthetic"][f"photo_{k}"][mode]
        assert (len(e), hashlib.sha256(e).hexdigest()) == (want["len"], want["sha256"]), (k, mode)
