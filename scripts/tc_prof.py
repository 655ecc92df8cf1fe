"""Phase shares of tile_cost_kernel (diagnostic; needs a -DHC_TC_PROF build via HC_LIB_PATH).

    HC_LIB_PATH=abvar/TCP/libhcodec.so python scripts/tc_prof.py [--streams 8192]
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
    buf = (ctypes.c_ulonglong * 4)()
    for it in range(3):
        work = hc.compress_adapt_batch(raw, offs, lens, widths, enc, eoffs, ecaps, elens, est,
                                       use_diff=not a.no_diff, work=work)
        torch.cuda.synchronize()
        L.hc_debug_tc_prof(ctypes.cast(buf, ctypes.c_void_p), 1)
    tot = sum(buf)
    names = ["load tile", "equality words", "candidates B<=128", "summaries + sync"]
    print({n: round(100 * v / tot, 1) for n, v in zip(names, buf)}, "cycles per tile (WG thread 0):",
          round(tot / (S * (a.side // 128) ** 2)))


if __name__ == "__main__":
    main()
