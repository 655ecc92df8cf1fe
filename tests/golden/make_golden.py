"""Regenerate tests/golden/ from the REFERENCE BINARY (oracle/_ref/huffman-codec, compiled from
/root/reference/src by `make -C oracle ref`). Run in the build container only:

    python tests/golden/make_golden.py

Writes
  digests.json       sha256 + size of the reference's output for
                       * the sample corpus data/*.raw x {-c, -c -m, -c -a, -c -m -a}
                         (the raw inputs stay in /root/reference; only digests are kept)
                       * synthetic inputs at 512x512, k = 0..3
                       * synthetic photo k=0 at 4096x4096, -c -a -w 4096 (and with -m)
  vectors.json       small complete vectors: input bytes, reference arguments, reference
                     output bytes (hex) for edge cases (runs around the 258 cut, last-byte rule,
                     empty / 1-byte inputs, all 256 symbols, deep Fibonacci trees, W/H not
                     multiples of the block size, W = H = 8, malformed streams and their exit
                     codes)
  corpus/*.huf       the reference's complete outputs for a few corpus files: decoding them
                     must give back the raw file (sha256 in digests.json), and re-encoding that
                     must give the .huf byte for byte
"""
import hashlib
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

DATA = "/root/reference/data"
MODES = {"c": ["-c"], "cm": ["-c", "-m"], "ca": ["-c", "-a"], "cma": ["-c", "-m", "-a"]}
CORPUS_HUF = [("hd01", "c"), ("hd01", "cm"), ("hd01", "ca"), ("hd01", "cma"), ("df1h", "cm"),
              ("df1h", "cma"), ("df1v", "c"), ("df1v", "ca"), ("hd01extra", "cma"),
              ("hd01double", "cm")]


def sha(b):
    return hashlib.sha256(b).hexdigest()


def ref(args, data, tmp):
    rc, out, err = O.run_ref(args, data, tmp, o2=True)
    return rc, out


def fib_stream(n_sym=24, total=60000):
    """symbols with Fibonacci-like frequencies, sorted ascending: a deep FGK tree"""
    f = [1, 1]
    while len(f) < n_sym:
        f.append(f[-1] + f[-2])
    out = []
    for s, c in enumerate(f):
        out += [s * 7 % 256] * c
        if len(out) > total:
            break
    return bytes(out[:total])


def edge_inputs():
    rng = np.random.default_rng(5)
    cases = {}
    cases["empty"] = b""
    cases["one_byte"] = b"\x07"
    cases["zero_byte"] = b"\x00"
    for L in (1, 2, 3, 4, 5, 257, 258, 259, 260, 515, 516, 517, 774, 775):
        cases[f"run{L}_final"] = b"\x05" * L
        cases[f"run{L}_then_x"] = b"\x05" * L + b"\x09"
        cases[f"zeros{L}_then_x"] = b"\x00" * L + b"\x01"
    cases["all256"] = bytes(range(256))
    cases["all256x4"] = bytes(range(256)) * 4
    cases["all256_rev"] = bytes(range(255, -1, -1)) * 3
    cases["random_1k"] = rng.integers(0, 256, 1000, dtype=np.uint8).tobytes()
    cases["random_runs"] = b"".join(bytes([int(rng.integers(0, 4))]) * int(rng.integers(1, 600))
                                     for _ in range(60))
    cases["two_symbols"] = bytes(rng.integers(0, 2, 5000, dtype=np.uint8))
    cases["fibonacci"] = fib_stream()
    cases["odd_len_4099"] = rng.integers(0, 16, 4099, dtype=np.uint8).tobytes()
    return cases


def matrix_inputs():
    """(name, bytes, width) for adaptive mode"""
    rng = np.random.default_rng(6)
    out = []
    out.append(("m8x8", rng.integers(0, 3, 64, dtype=np.uint8).tobytes(), 8))
    out.append(("m24x40", O.synth("photo", 3, 24, 40).tobytes(), 24))
    out.append(("m40x24", O.synth("grad", 1, 40, 24).tobytes(), 40))
    out.append(("m64x64_photo", O.synth("photo", 0, 64, 64).tobytes(), 64))
    out.append(("m100x37", rng.integers(0, 2, 3700, dtype=np.uint8).tobytes(), 100))
    out.append(("m33x129_runs", np.repeat(rng.integers(0, 3, 33 * 129 // 11 + 1, dtype=np.uint8),
                                          11)[:33 * 129].tobytes(), 33))
    out.append(("m7x20_small", bytes(140), 7))        # W < 8: status 12
    out.append(("m20x7_small", bytes(140), 20))       # H < 8: status 12
    out.append(("m10x9_bad", bytes(91), 10))          # size % W != 0: status 6
    return out


def malformed_streams(tmp):
    """(name, stream bytes) built from valid reference outputs by corruption"""
    base_raw = O.synth("photo", 1, 64, 64).tobytes()
    _, good = ref(["-c", "-m"], base_raw, tmp)
    _, good_a = ref(["-c", "-a", "-w", "64"], base_raw, tmp)
    out = []
    out.append(("short0", b""))
    out.append(("short8", good[:8]))
    out.append(("hdr_only", good[:9]))
    out.append(("trunc_half", good[: len(good) // 2]))
    out.append(("trunc_last", good[:-1]))
    big = bytearray(good)
    big[0:8] = (int.from_bytes(good[0:8], "little") + 5).to_bytes(8, "little")
    out.append(("count_plus5", bytes(big)))
    out.append(("count_huge", (1 << 40).to_bytes(8, "little") + good[8:]))
    extra = bytearray(good) + b"\xff\xff"
    out.append(("trailing_pad", bytes(extra)))
    flip = bytearray(good)
    flip[8] ^= 0x80
    out.append(("flag_flip_diff", bytes(flip)))
    out.append(("a_trunc", good_a[: len(good_a) * 2 // 3]))
    # adaptive payloads with forged headers, FGK-encoded through the oracle
    n = 64 * 64
    sym_ok = O.adapt(base_raw, 64, 64)[1]
    forged = {
        "a_hdr_short": sym_ok[:20],
        "a_dirs_missing": sym_ok[:24],
        "a_block_eof": sym_ok[:-5],
        "a_leftover": sym_ok + b"\x01\x02",
        "a_overshoot": sym_ok[:24 + 64] + b"\x07\x07\x07\xff" + sym_ok[24 + 64:],
    }
    for name, sym in forged.items():
        payload, nbits = O.fgk_encode(sym)
        stream = len(sym).to_bytes(8, "little") + bytes([0x40]) + payload
        out.append((name, stream))
    assert n == 4096
    return out


def main():
    os.makedirs(os.path.join(HERE, "corpus"), exist_ok=True)
    digests = {"corpus": {}, "synthetic": {}, "synthetic_4096": {}}
    vectors = {"compress": [], "adaptive": [], "decompress": []}
    with tempfile.TemporaryDirectory() as tmp:
        if os.path.isdir(DATA):
            for fn in sorted(os.listdir(DATA)):
                if not fn.endswith(".raw"):
                    continue
                name = fn[:-4]
                raw = open(os.path.join(DATA, fn), "rb").read()
                digests["corpus"][name] = {"raw_sha256": sha(raw), "raw_len": len(raw)}
                for m, args in MODES.items():
                    rc, out = ref(args, raw, tmp)
                    assert rc == 0
                    digests["corpus"][name][m] = {"sha256": sha(out), "len": len(out)}
                    if (name, m) in CORPUS_HUF:
                        with open(os.path.join(HERE, "corpus", f"{name}.{m}.huf"), "wb") as f:
                            f.write(out)
        for kind in ("photo", "grad", "noise"):
            for k in range(4):
                raw = O.synth(kind, k).tobytes()
                e = {"raw_sha256": sha(raw)}
                for m, args in MODES.items():
                    rc, out = ref(args, raw, tmp)
                    assert rc == 0
                    e[m] = {"sha256": sha(out), "len": len(out),
                            "count": int.from_bytes(out[:8], "little")}
                digests["synthetic"][f"{kind}_{k}"] = e
        raw = O.synth("photo", 0, 4096, 4096).tobytes()
        e = {"raw_sha256": sha(raw)}
        for m, args in (("ca", ["-c", "-a", "-w", "4096"]), ("cma", ["-c", "-m", "-a", "-w", "4096"])):
            rc, out = ref(args, raw, tmp)
            assert rc == 0
            e[m] = {"sha256": sha(out), "len": len(out), "count": int.from_bytes(out[:8], "little")}
        digests["synthetic_4096"]["photo_0"] = e

        for name, data in edge_inputs().items():
            for m in ("c", "cm"):
                rc, out = ref(MODES[m], data, tmp)
                vectors["compress"].append({"name": name, "mode": m, "input": data.hex(), "rc": rc,
                                            "output": out.hex()})
        for name, data, w in matrix_inputs():
            for m in ("ca", "cma"):
                rc, out = ref(MODES[m] + ["-w", str(w)], data, tmp)
                vectors["adaptive"].append({"name": name, "mode": m, "width": w, "input": data.hex(),
                                            "rc": rc, "output": out.hex()})
        for name, stream in malformed_streams(tmp):
            rc, out = ref(["-d"], stream, tmp)
            vectors["decompress"].append({"name": name, "input": stream.hex(), "rc": rc,
                                          "output": out.hex() if rc == 0 else ""})
    with open(os.path.join(HERE, "digests.json"), "w") as f:
        json.dump(digests, f, indent=1, sort_keys=True)
    with open(os.path.join(HERE, "vectors.json"), "w") as f:
        json.dump(vectors, f, indent=0)
    print("corpus", len(digests["corpus"]), "synthetic", len(digests["synthetic"]),
          "vectors", {k: len(v) for k, v in vectors.items()})


if __name__ == "__main__":
    main()
