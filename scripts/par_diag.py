"""Diagnostic: the parallel boundary pass on the 4096^2 photo streams (C4 / C4m): whether it ran,
fell back, and how many chunks par_fix re-ran (AMeta of the stream's workspace after a decode;
layout: hc_adapt.hip, par at byte 356, pfall 360, nsub 408, nchk 416, preruns 424)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "huffman-codec_amd", "python"))
import torch  # noqa: E402

import hcodec as hc  # noqa: E402

hc.use_debug_build(True)
dev = torch.device("cuda", 0)
W = 4096
N = W * W
for use_diff in (False, True):
    raw = torch.empty(N, dtype=torch.uint8, device=dev)
    hc.synth_batch("photo", 0, 1, W, W, raw, N)
    i64 = dict(dtype=torch.int64, device=dev)
    offs, lens, widths = torch.zeros(1, **i64), torch.full((1,), N, **i64), torch.full((1,), W, **i64)
    cap = hc.compress_bound(N, True)
    enc = torch.empty(cap, dtype=torch.uint8, device=dev)
    eoffs, ecaps, elens = torch.zeros(1, **i64), torch.full((1,), cap, **i64), torch.zeros(1, **i64)
    est = torch.zeros(1, dtype=torch.int32, device=dev)
    hc.compress_adapt_batch(raw, offs, lens, widths, enc, eoffs, ecaps, elens, est, use_diff=use_diff)
    back = torch.empty_like(raw)
    blens, bst = torch.zeros(1, **i64), torch.zeros(1, dtype=torch.int32, device=dev)
    work = hc.decompress_adapt_batch(enc, eoffs, elens, back, offs, lens, blens, bst)
    torch.cuda.synchronize()
    assert int(bst[0]) == 0 and torch.equal(back, raw)
    meta = work[:496].cpu().numpy()
    m64 = meta.view("uint64")
    m32 = meta.view("uint32")
    print(f"{'-c -a -m' if use_diff else '-c -a'}: parallel pass {m32[356 // 4]}, fallback {m32[360 // 4]},"
          f" sub-chunks {m64[408 // 8]}, chunks {m64[416 // 8]}, chunks re-run by par_fix {m64[424 // 8]}")
    d = m64[432 // 8:496 // 8]
    us = lambda c: f"{c / 2400:.0f} us"  # s_memtime: the shader clock, ~2.4 GHz
    print(f"  par_scan consumer: slot waits {us(d[0])}, tests {us(d[1])} (slow hits {us(d[2])}); sub-chunks"
          f" tested again {d[3]} (dense {d[7]}), skipped by the bitmap {d[4]}, fast hits {d[5]}, slow hits {d[6]}")
