"""Config C5 at full size on one GPU: 65536 photo 512x512 streams, -c -m, through the batched C ABI
(hc_compress_batch / hc_decompress_batch), the workload bench.py times.

Checked: every stream round-trips exactly and reports status 0; two encodes give the same
sizes; streams 0..3 equal the reference binary's digests (tests/golden/digests.json); 24 streams
spread over the batch (first, last, and across the middle) equal the oracle's encoding of the
same generated matrix byte for byte (oracle/hc_oracle.c, pinned to the reference in
tests/test_oracle.py); and the device pack of all encoded streams (hc_pack_batch, the step
before bench.py's RCCL gather) equals their concatenation. The RCCL gather itself needs more
than one GPU (covered on CPU by tests/test_dist.py).
"""
import hashlib

import pytest

pytestmark = pytest.mark.gpu

N = 262144
S = 65536


def test_c5_full_batch(gpu, hc, oracle_mod, digests):
    torch = gpu
    dev = "cuda"
    i64 = dict(dtype=torch.int64, device=dev)
    raw = torch.empty(S * N, dtype=torch.uint8, device=dev)
    hc.synth_batch("photo", 0, S, 512, 512, raw, N)
    offs = torch.arange(S, **i64) * N
    lens = torch.full((S,), N, **i64)
    cap = N + N // 2  # photo -c -m streams code to ~86 KB; a larger one would report 64
    enc = torch.empty(S * cap, dtype=torch.uint8, device=dev)
    eoffs = torch.arange(S, **i64) * cap
    ecaps = torch.full((S,), cap, **i64)
    elens = torch.zeros(S, **i64)
    st = torch.zeros(S, dtype=torch.int32, device=dev)
    hc.compress_batch(raw, offs, lens, enc, eoffs, ecaps, elens, st, use_diff=True)
    elens2 = torch.zeros_like(elens)
    st1 = torch.zeros_like(st)
    hc.compress_batch(raw, offs, lens, enc, eoffs, ecaps, elens2, st1, use_diff=True)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0 and int(st1.abs().sum()) == 0
    assert torch.equal(elens, elens2)

    # the reference's digests (photo k = 0..3) and the oracle on streams across the batch
    for k in range(4):
        e = enc[k * cap:k * cap + int(elens[k])].cpu().numpy().tobytes()
        want = digests["synthetic"]["photo_%d" % k]["cm"]
        assert (len(e), hashlib.sha256(e).hexdigest()) == (want["len"], want["sha256"]), k
    sample = sorted({0, 1, S - 1, S - 2} | {(S // 20) * j + 7 * j for j in range(20)})
    for k in sample:
        m = raw[k * N:(k + 1) * N].cpu().numpy().tobytes()
        assert m == oracle_mod.synth("photo", k).tobytes(), k
        ost, want = oracle_mod.compress(m, use_diff=True)
        got = enc[k * cap:k * cap + int(elens[k])].cpu().numpy().tobytes()
        assert ost == 0 and got == want, k

    # device pack of the encoded streams back to back (bench.py --gather packs the same way)
    total = int(elens.sum())
    packed = torch.empty(total, dtype=torch.uint8, device=dev)
    poffs = torch.cumsum(elens, 0) - elens
    hc.pack_batch(enc, eoffs, elens, packed, poffs)
    torch.cuda.synchronize()
    for k in (0, S // 2, S - 1):
        a, n = int(poffs[k]), int(elens[k])
        assert torch.equal(packed[a:a + n], enc[k * cap:k * cap + n]), k
    want_sum = 0
    ar = torch.arange(cap, device=dev).view(1, -1)
    for c0 in range(0, S, 2048):  # checksum of every encoded byte, in slices of the batch
        rows = enc.view(S, cap)[c0:c0 + 2048]
        want_sum += int((rows * (ar < elens[c0:c0 + 2048].view(-1, 1))).sum(dtype=torch.int64))
    assert int(packed.sum(dtype=torch.int64)) == want_sum
    del packed

    back = torch.empty_like(raw)
    blens = torch.zeros_like(lens)
    st2 = torch.zeros_like(st)
    hc.decompress_batch(enc, eoffs, elens, back, offs, lens, blens, st2)
    torch.cuda.synchronize()
    assert int(st2.abs().sum()) == 0
    assert torch.equal(blens, lens)
    assert torch.equal(back, raw)
