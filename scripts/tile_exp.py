"""A/B of adaptive-stage kernel variants on the A512 batch (8192 x 512^2 photo -c -a -m), in one
process: for each build directory given (each holding libhcodec_dbg.so), the stage clock's times
of `reps` encode + decode passes (median), and whether the encoded streams and the decoded
matrices equal those of the first build.

    python scripts/tile_exp.py [--reps 3] [--streams 8192] [--no-diff] dirA dirB ...
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "huffman-codec_amd", "python"))

import torch  # noqa: E402
import hcodec as hc  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--streams", type=int, default=8192)
    ap.add_argument("--side", type=int, default=512)
    ap.add_argument("--no-diff", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(dev)
    ref = None
    for d in args.dirs:
        path = os.path.join(d, "libhcodec_dbg.so")
        hc.DBG_LIB_PATH = path
        hc.LIB_PATH = path
        hc.use_debug_build(True)
        b = bench.AdaptBatch(torch, hc, dev, "photo", args.streams, not args.no_diff, args.side)
        times = {}
        try:
            for _ in range(args.reps):
                st = bench.adapt_stages(torch, hc, b, stream)
                hc.DBG_LIB_PATH = path  # (adapt_stages switches back to LIB_PATH, the same file)
                for direction in ("encode", "decode"):
                    for name, e in st[direction].items():
                        times.setdefault((direction, name), []).append(e["ms"])
        except Exception as ex:  # (a broken variant: report it, go on with the next)
            print(f"{d}: FAILED {type(ex).__name__}: {ex}", flush=True)
            del b
            torch.cuda.empty_cache()
            continue
        torch.cuda.synchronize(dev)
        enc_sig = (int(b.elens.sum()), int(b.est.abs().sum()),
                   int((b.enc.to(torch.int64) * (torch.arange(b.enc.numel(), device=dev) % 251 + 1)).sum()))
        ok_rt = bool(torch.equal(b.back, b.raw)) and int(b.bst.abs().sum()) == 0
        if ref is None:
            ref = enc_sig
        same = enc_sig == ref
        keep = ("tile_cost", "big_cost", "choose", "emit_tile", "fgk_encode", "fgk_decode", "bounds",
                "unblock_tile", "chunk_sum", "undiff")
        line = " ".join(f"{n}={statistics.median(v):.3f}" for (dd, n), v in times.items() if n in keep)
        print(f"{d}: {line} | enc_same={same} roundtrip={ok_rt}", flush=True)
        del b
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
