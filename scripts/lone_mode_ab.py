"""Encoder cache mode vs table mode (hc_debug_set_enc_tab) for lone streams (diagnostic): C2
(one 512x512 photo -c -m) and C4m (one 4096x4096 photo -c -a -m), kernel-inclusive wall time of
the batched calls on a resident input, and the encodings compared across modes.

    python scripts/lone_mode_ab.py
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
    i64 = dict(dtype=torch.int64, device=dev)
    for name, side, adapt, diff in (("C2", 512, False, True), ("C3-1", 512, False, False), ("C4m", 4096, True, True),
                                    ("C4", 4096, True, False)):
        N = side * side
        raw = torch.empty(N, dtype=torch.uint8, device=dev)
        hc.synth_batch("photo", 0, 1, side, side, raw, N)
        z = torch.zeros(1, **i64)
        lens = torch.tensor([N], **i64)
        cap = hc.compress_bound(N, adapt)
        enc = torch.empty(cap, dtype=torch.uint8, device=dev)
        caps = torch.tensor([cap], **i64)
        work = None
        if adapt:
            work = torch.empty(int(hc.lib().hc_adapt_compress_work_bound(N, 1)), dtype=torch.uint8, device=dev)
        res, outs = {}, {}
        for mask in (1, 2, 1, 2):
            hc.debug_set_enc_tab(mask)
            elens = torch.zeros(1, **i64)
            est = torch.zeros(1, dtype=torch.int32, device=dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if adapt:
                hc.compress_adapt_batch(raw, z, lens, torch.tensor([side], **i64), enc, z, caps, elens, est,
                                        use_diff=diff, work=work)
            else:
                hc.compress_batch(raw, z, lens, enc, z, caps, elens, est, use_diff=diff)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
            assert int(est[0]) == 0
            res.setdefault(mask, []).append(ms)
            outs[mask] = enc[:int(elens[0])].cpu().numpy().tobytes()
        hc.debug_set_enc_tab(0)
        print(name, {("cache" if m == 1 else "tables"): round(min(v), 2) for m, v in res.items()},
              "identical" if outs[1] == outs[2] else "DIFFER", flush=True)


if __name__ == "__main__":
    main()
