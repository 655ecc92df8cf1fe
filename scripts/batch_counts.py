"""Event counts of the FGK kernels' batched paths per stream (diagnostic).

Needs a library built with -DHC_PROF -DHC_COUNT (hc_fgk.hip HC_CNT): lane i of every wave's
accumulator counts event i; the counts land where path_prof.py's cycle sums do.
    bash scripts/build_rel.sh CNT -DHC_PROF -DHC_COUNT
    HC_LIB_PATH=abvar/CNT/libhcodec.so python scripts/batch_counts.py --kind grad
Encoder (code_all_batch): 1 batch steps, 2 symbols coded alone, 3 retests, 4 retests skipped
(failure not plausibly false), 5 failing symbol was a miss, 6 retests that moved jf on.
Decoder (decode_batch): 1 batch steps, 2 batches ending early, 3 retests, 4 skipped, 5 ended at a
non-leaf entry, 6 retests that moved jf on.
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "huffman-codec_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=1024)
    ap.add_argument("--kind", default="grad")
    ap.add_argument("--no-diff", action="store_true")
    args = ap.parse_args()
    import torch
    import hcodec as hc
    L = hc.lib()
    L.hc_debug_set_trace.argtypes = [ctypes.c_void_p]
    S, N = args.streams, 512 * 512
    dev = torch.device("cuda", 0)
    raw = torch.empty(S * N, dtype=torch.uint8, device=dev)
    hc.synth_batch(args.kind, 0, S, 512, 512, raw, N)
    i64 = dict(dtype=torch.int64, device=dev)
    offs = torch.arange(S, **i64) * N
    lens = torch.full((S,), N, **i64)
    cap = 2 * N + 4096
    enc = torch.empty(S * cap, dtype=torch.uint8, device=dev)
    eoffs = torch.arange(S, **i64) * cap
    ecaps = torch.full((S,), cap, **i64)
    elens = torch.zeros(S, **i64)
    est = torch.zeros(S, dtype=torch.int32, device=dev)
    back = torch.empty_like(raw)
    blens = torch.zeros_like(lens)
    bst = torch.zeros_like(est)
    trace = torch.zeros(8 * S, **i64)
    assert L.hc_debug_set_trace(ctypes.c_void_p(trace.data_ptr())) == 0
    try:
        hc.compress_batch(raw, offs, lens, enc, eoffs, ecaps, elens, est, use_diff=not args.no_diff)
        torch.cuda.synchronize()
        e = trace.view(S, 8).double().mean(0).cpu().tolist()
        trace.zero_()
        hc.decompress_batch(enc, eoffs, elens, back, offs, lens, blens, bst)
        torch.cuda.synchronize()
        d = trace.view(S, 8).double().mean(0).cpu().tolist()
    finally:
        L.hc_debug_set_trace(ctypes.c_void_p(0))
    ok = bool(torch.equal(back, raw)) and int((est != 0).sum()) == 0
    print(f"{args.kind} {'-c' if args.no_diff else '-c -m'} {S} streams, round trip {'exact' if ok else 'FAILED'}")
    print("encode per stream: steps %.1f alone %.1f retests %.1f skipped %.1f miss %.1f moved %.1f" % tuple(e[1:7]))
    print("decode per stream: steps %.1f early %.1f retests %.1f skipped %.1f nonleaf %.1f moved %.1f" % tuple(d[1:7]))


if __name__ == "__main__":
    main()
