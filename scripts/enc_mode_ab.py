"""Encoder cache mode vs table mode (hc_debug_set_enc_tab), kernel time of the batched encode
on synthetic 512x512 batches (diagnostic).

    python scripts/enc_mode_ab.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "huffman-codec_amd", "python"))


def main():
    import torch
    import hcodec as hc
    hc.use_debug_build(True)  # hc_debug_set_enc_tab: debug build only
    dev = torch.device("cuda", 0)
    N = 512 * 512
    cases = [("photo -c", "photo", 4096, False), ("photo -c 8192", "photo", 8192, False),
             ("photo -c -m", "photo", 8192, True), ("noise -c -m", "noise", 2048, True),
             ("grad -c", "grad", 8192, False)]
    for name, kind, S, diff in cases:
        raw = torch.empty(S * N, dtype=torch.uint8, device=dev)
        hc.synth_batch(kind, 0, S, 512, 512, raw, N)
        i64 = dict(dtype=torch.int64, device=dev)
        offs = torch.arange(S, **i64) * N
        lens = torch.full((S,), N, **i64)
        cap = 2 * N + 4096
        enc = torch.empty(S * cap, dtype=torch.uint8, device=dev)
        eoffs = torch.arange(S, **i64) * cap
        ecaps = torch.full((S,), cap, **i64)
        res = {}
        outs = {}
        for mask in (1, 2, 0, 1, 2, 0):
            hc.debug_set_enc_tab(mask)
            elens = torch.zeros(S, **i64)
            est = torch.zeros(S, dtype=torch.int32, device=dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            hc.compress_batch(raw, offs, lens, enc, eoffs, ecaps, elens, est, use_diff=diff)
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(mask, []).append(e0.elapsed_time(e1))
            outs[mask] = (int(elens.sum()), int((est != 0).sum()))
        hc.debug_set_enc_tab(0)
        print(f"{name:16s} streams {S:5d}  cache {min(res[1]):8.2f} ms  tables {min(res[2]):8.2f} ms  "
              f"auto {min(res[0]):8.2f} ms  same bytes {outs[0] == outs[1] == outs[2]}", flush=True)
        del raw, enc


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def adaptive():
    """the adaptive configs (symbol streams, bit 2): A512 and C4 / C4m"""
    import torch
    import hcodec as hc
    hc.use_debug_build(True)  # hc_debug_set_enc_tab: debug build only
    dev = torch.device("cuda", 0)
    for name, S, side, diff in (("A512 -a -m", 8192, 512, True), ("A512 -a", 8192, 512, False),
                                ("C4 -a", 1, 4096, False), ("C4m -a -m", 1, 4096, True)):
        N = side * side
        raw = torch.empty(S * N, dtype=torch.uint8, device=dev)
        hc.synth_batch("photo", 0, S, side, side, raw, N)
        i64 = dict(dtype=torch.int64, device=dev)
        offs = torch.arange(S, **i64) * N
        lens = torch.full((S,), N, **i64)
        widths = torch.full((S,), side, **i64)
        cap = (hc.compress_bound(N, True) + 255) // 256 * 256
        enc = torch.empty(S * cap, dtype=torch.uint8, device=dev)
        eoffs = torch.arange(S, **i64) * cap
        ecaps = torch.full((S,), cap, **i64)
        work = None
        res, outs = {}, {}
        for mask in (1, 2, 0):
            hc.debug_set_enc_tab(mask)
            elens = torch.zeros(S, **i64)
            est = torch.zeros(S, dtype=torch.int32, device=dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            work = hc.compress_adapt_batch(raw, offs, lens, widths, enc, eoffs, ecaps, elens, est, use_diff=diff,
                                           work=work)
            e1.record()
            torch.cuda.synchronize()
            res[mask] = e0.elapsed_time(e1)
            outs[mask] = (int(elens.sum()), int((est != 0).sum()))
        hc.debug_set_enc_tab(0)
        print(f"{name:16s} streams {S:5d}  cache {res[1]:9.2f} ms  tables {res[2]:9.2f} ms  auto {res[0]:9.2f} ms  "
              f"same bytes {outs[0] == outs[1] == outs[2]}", flush=True)
        del raw, enc, work


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "adaptive":
    adaptive()
