"""PCIe-inclusive rate of the host-buffer boundary (diagnostic): hc_compress_host_batch /
hc_decompress_host_batch on S synthetic photo 512x512 streams that sit in pageable host memory
(one numpy buffer, streams back to back), timed around the C calls only (the pipelined
sub-batches: pinned staging, H2D, kernels, D2H, copy out). Also the batched adaptive pair.

    python scripts/host_batch_rate.py [--streams 8192] [--no-diff]
"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "huffman-codec_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=8192)
    ap.add_argument("--no-diff", action="store_true")
    args = ap.parse_args()
    import numpy as np
    import torch
    import hcodec as hc
    S, N = args.streams, 512 * 512
    diff = not args.no_diff
    dev = torch.device("cuda", 0)
    d = torch.empty(S * N, dtype=torch.uint8, device=dev)
    hc.synth_batch("photo", 0, S, 512, 512, d, N)
    raw = d.cpu().numpy()
    del d
    torch.cuda.empty_cache()
    L = hc.lib()
    P = ctypes.c_void_p * S
    U = ctypes.c_uint64 * S

    def ptrs(buf, stride):
        base = buf.ctypes.data
        return vp(P(*[base + i * stride for i in range(S)]))

    def vp(arr):
        return ctypes.cast(arr, ctypes.c_void_p)

    def run(adapt):
        cap = hc.compress_bound(N, adapt)
        enc = np.empty(S * cap, dtype=np.uint8)
        back = np.empty_like(raw)
        lens, caps, olens = U(*([N] * S)), U(*([cap] * S)), U()
        st = (ctypes.c_int32 * S)()
        flags = hc.HC_FLAG_DIFF if diff else 0
        t0 = time.perf_counter()
        if adapt:
            widths = U(*([512] * S))
            rc = L.hc_compress_adapt_host_batch(ptrs(raw, N), vp(lens), vp(widths), S, flags, ptrs(enc, cap), vp(caps),
                                                vp(olens), vp(st))
        else:
            rc = L.hc_compress_host_batch(ptrs(raw, N), vp(lens), S, flags, ptrs(enc, cap), vp(caps), vp(olens), vp(st))
        te = time.perf_counter() - t0
        assert rc == 0 and all(s == 0 for s in st)
        elens = U(*olens)
        dl, dst = U(), (ctypes.c_int32 * S)()
        t0 = time.perf_counter()
        ncap = U(*([N] * S))
        rc = L.hc_decompress_host_batch(ptrs(enc, cap), vp(elens), S, ptrs(back, N), vp(ncap), vp(dl), vp(dst))
        td = time.perf_counter() - t0
        assert rc == 0 and all(s == 0 for s in dst)
        assert np.array_equal(back, raw)
        gib = S * N / 2**30
        mode = ("-c -a" if adapt else "-c") + (" -m" if diff else "")
        print(f"{S} x 512x512 photo {mode}, host buffers: encode {te * 1e3:.1f} ms ({gib / te:.2f} GiB/s), "
              f"decode {td * 1e3:.1f} ms ({gib / td:.2f} GiB/s), round trip {gib / (te + td):.2f} GiB/s", flush=True)

    for adapt in (False, True):
        run(adapt)
        run(adapt)


if __name__ == "__main__":
    main()
