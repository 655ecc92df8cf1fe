"""Where the FGK kernels spend their cycles, by code path (diagnostic).

Needs a library built with -DHC_PROF (hc_fgk.hip: HC_PROF_BEGIN/END): every wave sums the
s_memtime cycles of each region into lane i of an accumulator and stores lanes 0..7 at
g_trace[8 * stream + i] (lane 0 = the wave's whole life). s_memtime itself costs cycles, so
the shares are indicative, not exact.

    make -C huffman-codec_amd lib/libhcodec.so EXTRA=-DHC_PROF -B && cp ... abvar/P/
    HC_LIB_PATH=abvar/P/libhcodec.so python scripts/path_prof.py [--streams 8192]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "huffman-codec_amd", "python"))

ENC = {1: "miss (chase, insert, update, push)", 5: "  of which: chase", 6: "  of which: update (walk)",
       2: "walk after a failed leader test", 3: "record pack", 4: "MNP-5 chunk pass",
       7: "  of which (any walk): cache scan per swap"}
# encoder table mode (code_all_tab; --enc-tab 2)
TAB = {1: "miss (not in the tables)", 6: "  of which: chase", 7: "  of which: update (walk)",
       2: "walk after a failed leader test", 3: "record pack", 4: "MNP-5 chunk pass", 5: "level table rebuild"}
DEC = {1: "walk after a failed leader test", 2: "long code descent / NYT", 3: "update after descent / NYT",
       4: "RLE + diff revert", 5: "level table rebuild", 6: "batch step (narrow / wide)"}


def report(name, names, tr):
    tot = tr[:, 0].sum()
    print(f"{name}: mean wave life {tr[:, 0].mean():.4g} cycles", flush=True)
    rest = tot
    for i, what in names.items():
        share = tr[:, i].sum() / tot
        if not what.startswith("  of which"):
            rest -= tr[:, i].sum()
        print(f"  {what:36s} {100 * share:5.1f} %")
    print(f"  {'hot loop and the rest':36s} {100 * rest / tot:5.1f} %", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=8192)
    ap.add_argument("--kind", default="photo")
    ap.add_argument("--no-diff", action="store_true")
    ap.add_argument("--enc-tab", type=int, default=0, help="encoder mode: 0 auto, 1 cache, 2 tables")
    args = ap.parse_args()
    import torch
    import hcodec as hc
    L = hc.use_debug_build(True)  # hc_debug_set_trace: debug build only
    L.hc_debug_set_trace.argtypes = [ctypes.c_void_p]
    S, N = args.streams, 512 * 512
    dev = torch.device("cuda", 0)
    raw = torch.empty(S * N, dtype=torch.uint8, device=dev)
    hc.synth_batch(args.kind, 0, S, 512, 512, raw, N)
    offs = torch.arange(S, dtype=torch.int64, device=dev) * N
    lens = torch.full((S,), N, dtype=torch.int64, device=dev)
    cap = 2 * N + 4096
    enc = torch.empty(S * cap, dtype=torch.uint8, device=dev)
    eoffs = torch.arange(S, dtype=torch.int64, device=dev) * cap
    ecaps = torch.full((S,), cap, dtype=torch.int64, device=dev)
    elens = torch.zeros(S, dtype=torch.int64, device=dev)
    est = torch.zeros(S, dtype=torch.int32, device=dev)
    back = torch.empty_like(raw)
    blens = torch.zeros_like(lens)
    bst = torch.zeros_like(est)
    trace = torch.zeros(8 * S, dtype=torch.int64, device=dev)
    diff = not args.no_diff
    hc.debug_set_enc_tab(args.enc_tab)
    assert L.hc_debug_set_trace(ctypes.c_void_p(trace.data_ptr())) == 0
    try:
        hc.compress_batch(raw, offs, lens, enc, eoffs, ecaps, elens, est, use_diff=diff)
        torch.cuda.synchronize()
        report("encode_kernel", TAB if args.enc_tab == 2 else ENC, trace.view(S, 8).double().cpu().numpy())
        trace.zero_()
        hc.decompress_batch(enc, eoffs, elens, back, offs, lens, blens, bst)
        torch.cuda.synchronize()
        report("decode_kernel", DEC, trace.view(S, 8).double().cpu().numpy())
    finally:
        L.hc_debug_set_trace(ctypes.c_void_p(0))
        torch.cuda.synchronize()
    assert torch.equal(back, raw)


if __name__ == "__main__":
    main()
