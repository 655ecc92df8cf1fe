"""The oracle (oracle/hc_oracle.c, a C restatement) pinned against the reference.

Pinning: every golden vector and digest in tests/golden/ was produced by the reference binary
itself (oracle/_ref/huffman-codec, built from /root/reference/src; see make_golden.py). When
/root/reference is present (build container) the oracle is also checked against the reference
corpus data/*.raw and against the freshly built reference binary.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import REF_DATA

MODES = {"c": (False, False), "cm": (True, False), "ca": (False, True), "cma": (True, True)}


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_synthetic_generator_matches_survey(oracle_mod, digests):
    for name, e in digests["synthetic"].items():
        kind, k = name.split("_")
        assert sha(oracle_mod.synth(kind, int(k)).tobytes()) == e["raw_sha256"], name


@pytest.mark.parametrize("kind", ["photo", "grad", "noise"])
def test_oracle_compress_synthetic_digests(oracle_mod, digests, kind):
    for k in range(2):
        raw = oracle_mod.synth(kind, k).tobytes()
        e = digests["synthetic"][f"{kind}_{k}"]
        for m, (d, a) in MODES.items():
            if kind == "noise" and a:
                continue  # slow in the pointer-tree oracle; covered by test_oracle_vectors
            st, out = oracle_mod.compress(raw, d, a, 512)
            assert st == 0
            assert (len(out), sha(out)) == (e[m]["len"], e[m]["sha256"]), (kind, k, m)
            st, back = oracle_mod.decompress(out)
            assert st == 0 and back == raw


def test_oracle_vectors_compress(oracle_mod, vectors):
    for v in vectors["compress"]:
        d, a = MODES[v["mode"]]
        st, out = oracle_mod.compress(bytes.fromhex(v["input"]), d, a, 512)
        assert st == v["rc"], v["name"]
        assert out.hex() == v["output"], (v["name"], v["mode"])


def test_oracle_vectors_adaptive(oracle_mod, vectors):
    for v in vectors["adaptive"]:
        d, a = MODES[v["mode"]]
        st, out = oracle_mod.compress(bytes.fromhex(v["input"]), d, a, v["width"])
        assert st == v["rc"], v["name"]
        assert out.hex() == v["output"], (v["name"], v["mode"])


def test_oracle_vectors_decompress(oracle_mod, vectors):
    for v in vectors["decompress"]:
        st, out = oracle_mod.decompress(bytes.fromhex(v["input"]))
        assert st == v["rc"], v["name"]
        if st == 0:
            assert out.hex() == v["output"], v["name"]


def test_oracle_corpus_huf_roundtrip(oracle_mod, digests):
    gdir = os.path.join(os.path.dirname(__file__), "golden", "corpus")
    for fn in sorted(os.listdir(gdir)):
        name, m, _ = fn.split(".")
        huf = open(os.path.join(gdir, fn), "rb").read()
        st, raw = oracle_mod.decompress(huf)
        assert st == 0
        assert sha(raw) == digests["corpus"][name]["raw_sha256"], fn
        d, a = MODES[m]
        st, again = oracle_mod.compress(raw, d, a, 512)
        assert st == 0 and again == huf, fn


@pytest.mark.skipif(not os.path.isdir(REF_DATA), reason="reference corpus not present (GPU box)")
def test_oracle_corpus_digests(oracle_mod, digests):
    for name in ("hd01", "df1hvx", "hd01extra", "hd12"):
        raw = open(os.path.join(REF_DATA, name + ".raw"), "rb").read()
        assert sha(raw) == digests["corpus"][name]["raw_sha256"]
        for m, (d, a) in MODES.items():
            st, out = oracle_mod.compress(raw, d, a, 512)
            assert st == 0
            e = digests["corpus"][name][m]
            assert (len(out), sha(out)) == (e["len"], e["sha256"]), (name, m)


def test_slot_form_equals_pointer_form(oracle_mod):
    rng = np.random.default_rng(1)
    streams = [oracle_mod.rle(oracle_mod.diff(oracle_mod.synth("photo", 3, 128, 128))),
               rng.integers(0, 256, 20000, dtype=np.uint8).tobytes(),
               rng.geometric(0.05, 20000).clip(0, 255).astype(np.uint8).tobytes(),
               bytes(rng.integers(0, 3, 5000, dtype=np.uint8))]
    for s in streams:
        a = oracle_mod.fgk_encode(s)
        b = oracle_mod.fgk_encode(s, slot_form=True)
        assert a == b
        st, back = oracle_mod.fgk_decode(b[0], len(s), slot_form=True)
        assert st == 0 and back == s


def _rle_closed_form(data):
    """the MNP-5 output as a function of the runs of the input"""
    out = bytearray()
    i, n = 0, len(data)
    while i < n:
        j = i
        while j < n and data[j] == data[i]:
            j += 1
        b, L = data[i], j - i
        final = j == n
        if final:
            L -= 1
        out += bytes([b, b, b, 255]) * (L // 258)
        r = L % 258
        if r in (1, 2):
            out += bytes([b]) * r
        elif r >= 3:
            out += bytes([b, b, b, r - 3])
        if final:
            out.append(b)
        i = j
    return bytes(out)


def test_rle_closed_form_and_roundtrip(oracle_mod):
    rng = np.random.default_rng(2)
    for t in range(300):
        nruns = int(rng.integers(1, 12))
        data = b"".join(bytes([int(rng.integers(0, 3))]) * int(rng.choice([1, 2, 3, 4, 257, 258, 259, 516, 517,
                                                                             int(rng.integers(1, 800))]))
                        for _ in range(nruns))
        enc = oracle_mod.rle(data)
        assert enc == _rle_closed_form(data), t
        assert oracle_mod.unrle(enc) == data


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(os.path.dirname(__file__)), "oracle",
                                                    "_ref", "huffman-codec")),
                    reason="reference binary not built")
def test_oracle_matches_reference_binary_random(oracle_mod, tmp_path):
    rng = np.random.default_rng(3)
    for t in range(6):
        n = int(rng.integers(0, 3000))
        data = bytes(rng.integers(0, int(rng.integers(1, 256)) + 1, n, dtype=np.uint16).astype(np.uint8))
        for m, args in (("c", ["-c"]), ("cm", ["-c", "-m"])):
            rc, ref, _ = oracle_mod.run_ref(args, data, str(tmp_path))
            st, out = oracle_mod.compress(data, m == "cm", False, 512)
            assert rc == st == 0 and ref == out
