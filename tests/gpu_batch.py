"""Helpers for GPU tests: pack byte strings into one device buffer and run the batch C ABI."""
import numpy as np


def align(x, a=16):
    return (x + a - 1) // a * a


def pack(torch, blobs, caps=None):
    """-> (device uint8 buffer, offs int64, lens int64) with 16-byte aligned stream starts"""
    lens = [len(b) for b in blobs]
    caps = caps if caps is not None else lens
    offs, o = [], 0
    for c in caps:
        offs.append(o)
        o = align(o + max(c, 1))
    host = np.zeros(max(o, 16), dtype=np.uint8)
    for off, b in zip(offs, blobs):
        if len(b):
            host[off:off + len(b)] = np.frombuffer(bytes(b), dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    t = lambda v: torch.tensor(v, dtype=torch.int64, device="cuda")
    return dev, t(offs), t(lens), t(list(caps))


def unpack(torch, buf, offs, lens):
    h = buf.cpu().numpy()
    o = offs.cpu().tolist()
    n = lens.cpu().tolist()
    return [h[a:a + b].tobytes() for a, b in zip(o, n)]


def compress_batch(hc, torch, raws, use_diff, cap_fn=None):
    din, ioffs, ilens, _ = pack(torch, raws)
    caps = [cap_fn(len(r)) if cap_fn else hc.compress_bound(len(r)) for r in raws]
    dout, ooffs, _, ocaps = pack(torch, [b""] * len(raws), caps)
    olens = torch.zeros(len(raws), dtype=torch.int64, device="cuda")
    st = torch.full((len(raws),), -1, dtype=torch.int32, device="cuda")
    hc.compress_batch(din, ioffs, ilens, dout, ooffs, ocaps, olens, st, use_diff=use_diff)
    torch.cuda.synchronize()
    return st.cpu().tolist(), unpack(torch, dout, ooffs, olens), olens.cpu().tolist()


def decompress_batch(hc, torch, encs, caps):
    din, ioffs, ilens, _ = pack(torch, encs)
    dout, ooffs, _, ocaps = pack(torch, [b""] * len(encs), caps)
    olens = torch.zeros(len(encs), dtype=torch.int64, device="cuda")
    st = torch.full((len(encs),), -1, dtype=torch.int32, device="cuda")
    hc.decompress_batch(din, ioffs, ilens, dout, ooffs, ocaps, olens, st)
    torch.cuda.synchronize()
    return st.cpu().tolist(), unpack(torch, dout, ooffs, olens), olens.cpu().tolist()


def compress_adapt_batch(hc, torch, raws, widths, use_diff, caps=None):
    din, ioffs, ilens, _ = pack(torch, raws)
    caps = caps if caps is not None else [hc.compress_bound(len(r), True) for r in raws]
    dout, ooffs, _, ocaps = pack(torch, [b""] * len(raws), caps)
    w = torch.tensor(list(widths), dtype=torch.int64, device="cuda")
    olens = torch.zeros(len(raws), dtype=torch.int64, device="cuda")
    st = torch.full((len(raws),), -1, dtype=torch.int32, device="cuda")
    hc.compress_adapt_batch(din, ioffs, ilens, w, dout, ooffs, ocaps, olens, st, use_diff=use_diff)
    torch.cuda.synchronize()
    return st.cpu().tolist(), unpack(torch, dout, ooffs, olens), olens.cpu().tolist()


def decompress_adapt_batch(hc, torch, encs, caps):
    din, ioffs, ilens, _ = pack(torch, encs)
    dout, ooffs, _, ocaps = pack(torch, [b""] * len(encs), caps)
    olens = torch.zeros(len(encs), dtype=torch.int64, device="cuda")
    st = torch.full((len(encs),), -1, dtype=torch.int32, device="cuda")
    hc.decompress_adapt_batch(din, ioffs, ilens, dout, ooffs, ocaps, olens, st)
    torch.cuda.synchronize()
    return st.cpu().tolist(), unpack(torch, dout, ooffs, olens), olens.cpu().tolist()
