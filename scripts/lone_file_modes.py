"""Single-buffer API (the CLI's path) on one real file, per encoder mode (diagnostic; debug build):
encode and decode wall time of hc_compress / hc_decompress in a warm process, median of 7.

    python scripts/lone_file_modes.py FILE.raw [--no-diff]
    (hd01.raw: decode tests/golden/corpus/hd01.cm.huf with the reference binary first, as bench.py's C1 does)
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "huffman-codec_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--no-diff", action="store_true")
    a = ap.parse_args()
    import hcodec as hc
    hc.use_debug_build(True)
    for path in a.paths:
        run(hc, path, a)


def run(hc, path, a):
    data = open(path, "rb").read()
    ref = None
    print(path, flush=True)
    for mode, name in ((0, "vote"), (1, "cache"), (2, "tables")):
        hc.debug_set_enc_tab(mode)
        enc_t, dec_t = [], []
        for _ in range(7):
            t0 = time.perf_counter()
            st, enc = hc.compress(data, use_diff=not a.no_diff)
            t1 = time.perf_counter()
            st2, back = hc.decompress(enc)
            t2 = time.perf_counter()
            enc_t.append(1e3 * (t1 - t0))
            dec_t.append(1e3 * (t2 - t1))
        assert st == 0 and st2 == 0 and back == data
        ref = ref or enc
        print(f"{name:6s} encode {statistics.median(enc_t):8.2f} ms  decode {statistics.median(dec_t):8.2f} ms"
              f"  bytes {len(enc)} same={enc == ref}", flush=True)
    hc.debug_set_enc_tab(0)


if __name__ == "__main__":
    main()
