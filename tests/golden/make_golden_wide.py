"""Add the "wide" goldens to tests/golden/digests.json from the REFERENCE BINARY
(oracle/_ref/huffman-codec-O2, byte-identical to the Makefile build). Build container only:

    python tests/golden/make_golden_wide.py

Non-adaptive inputs past the narrow FGK layout's 2^22 - 2 symbol limit. The encoder picks the
wide tree when n + n/3 + 2 > 2^22 - 2 (any raw input over ~3.1 MB), the decoder when the
stream's count exceeds 2^22 - 2, so these are the only inputs that reach
encode_kernel<true, SRC_RAW | SRC_RAW_DIFF> and decode_kernel<true, DST_RAW>
(huffman-codec_amd/csrc/hc_fgk.hip). Synthetic inputs at
  2048x2048 photo / grad / noise, k = 0   (wide encode; noise -c also a wide decode)
  4096x4096 photo, k = 0                   (wide encode and decode: ~12.9 M symbols)
in modes -c and -c -m. Only digests, sizes and counts are stored (writes key "wide").
"""
import hashlib
import json
import os
import sys
import tempfile
from concurrent.futures import ProcessPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

CASES = [("photo", 0, 2048), ("grad", 0, 2048), ("noise", 0, 2048), ("photo", 0, 4096)]
MODES = {"c": ["-c"], "cm": ["-c", "-m"]}


def one(job):
    kind, k, side, mode = job
    raw = O.synth(kind, k, side, side).tobytes()
    with tempfile.TemporaryDirectory() as tmp:
        rc, out, _ = O.run_ref(MODES[mode], raw, tmp, o2=True)
    assert rc == 0, job
    return job, hashlib.sha256(raw).hexdigest(), {
        "sha256": hashlib.sha256(out).hexdigest(), "len": len(out),
        "count": int.from_bytes(out[:8], "little")}


def main():
    path = os.path.join(HERE, "digests.json")
    with open(path) as f:
        digests = json.load(f)
    jobs = [(kind, k, side, m) for kind, k, side in CASES for m in MODES]
    wide = {}
    with ProcessPoolExecutor(4) as ex:
        for (kind, k, side, m), raw_sha, e in ex.map(one, jobs):
            d = wide.setdefault(f"{kind}_{k}_{side}", {"raw_sha256": raw_sha, "side": side})
            d[m] = e
            print(kind, side, m, e, flush=True)
    digests["wide"] = wide
    with open(path, "w") as f:
        json.dump(digests, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
