"""Phase shares of tile_cost_kernel and emit_tile_kernel (diagnostic; needs a -DHC_TC_PROF build,
scripts/build_var.sh TCP -DHC_TC_PROF, loaded through HC_LIB_PATH).

    HC_LIB_PATH=abvar/TCP/libhcodec_dbg.so python scripts/tc_prof.py [--streams 8192]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "huffman-codec_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=8192)
    ap.add_argument("--side", type=int, default=512)
    ap.add_argument("--no-diff", action="store_true")
    a = ap.parse_args()
    import torch
    import hcodec as hc
    L = hc.lib()
    L.hc_debug_tc_prof.argtypes = [ctypes.c_void_p, ctypes.c_int]
    S, N = a.streams, a.side * a.side
    dev = torch.device("cuda", 0)
    raw = torch.empty(S * N, dtype=torch.uint8, device=dev)
    hc.synth_batch("photo", 0, S, a.side, a.side, raw, N)
    i64 = dict(dtype=torch.int64, device=dev)
    offs = torch.arange(S, **i64) * N
    lens = torch.full((S,), N, **i64)
    widths = torch.full((S,), a.side, **i64)
    cap = 2 * N + 4096
    enc = torch.empty(S * cap, dtype=torch.uint8, device=dev)
    eoffs = torch.arange(S, **i64) * cap
    ecaps = torch.full((S,), cap, **i64)
    elens = torch.zeros(S, **i64)
    est = torch.zeros(S, dtype=torch.int32, device=dev)
    work = None
    buf = (ctypes.c_ulonglong * 16)()
    for it in range(3):
        work = hc.compress_adapt_batch(raw, offs, lens, widths, enc, eoffs, ecaps, elens, est,
                                       use_diff=not a.no_diff, work=work)
        torch.cuda.synchronize()
        L.hc_debug_tc_prof(ctypes.cast(buf, ctypes.c_void_p), 1)
    tiles = S * (a.side // 128) ** 2
    for name, lo, phases in (("tile_cost", 0, ["put barrier", "put load wait", "put diff+store", "equality words",
                                               "candidates B<=128", "summaries"]),
                             ("emit_tile", 8, ["put barrier", "put load wait", "put diff+store", "emit"])):
        vals = list(buf[lo:lo + len(phases)])
        tot = sum(vals) or 1
        print(name, {n: round(100 * v / tot, 1) for n, v in zip(phases, vals)},
              "cycles per tile (WG thread 0):", round(tot / tiles))

if __name__ == "__main__":
    main()
