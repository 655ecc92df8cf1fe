"""An adaptive (-c -a -m) stream at real size past 4 GiB (opt-in: HC_HUGE_ADAPT=1, a few minutes,
most of it the oracle on the host).

The reference's adaptive header carries u64 W / H / B and revertAdaptRLE has no size limit
(headers.cpp:18-105, transform.cpp:330-361). A 65536 x 65600 gradient matrix (4.30 GB, more
than 2^32 bytes) is generated in HBM, coded with the batched adaptive API (64-bit block offsets
and starts, the diff model over > 2^32 bytes, the parallel block-boundary pass at its real
threshold), compared byte for byte with the oracle's encoding of the same matrix, and decoded
back exactly. The gradient keeps the FGK symbol count moderate (runs collapse under the diff
model). Log: profiles/r03_huge_adapt.log.
"""
import hashlib
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(1100)
@pytest.mark.skipif(os.environ.get("HC_HUGE_ADAPT") != "1", reason="opt-in: a few minutes (oracle on the host)")
def test_huge_adaptive_stream(gpu, hc, oracle_mod):
    torch = gpu
    W, H = 65600, 65536
    N = W * H
    assert N > 1 << 32
    dev = torch.device("cuda", 0)
    raw = torch.empty(N, dtype=torch.uint8, device=dev)
    hc.synth_batch("grad", 0, 1, W, H, raw, N)
    i64 = dict(dtype=torch.int64, device=dev)
    offs, lens, widths = torch.zeros(1, **i64), torch.full((1,), N, **i64), torch.full((1,), W, **i64)
    cap = 1 << 30
    enc = torch.zeros(cap, dtype=torch.uint8, device=dev)
    eoffs, ecaps, elens = torch.zeros(1, **i64), torch.full((1,), cap, **i64), torch.zeros(1, **i64)
    est = torch.full((1,), -1, dtype=torch.int32, device=dev)
    t0 = time.time()
    work = hc.compress_adapt_batch(raw, offs, lens, widths, enc, eoffs, ecaps, elens, est, use_diff=True)
    torch.cuda.synchronize()
    del work
    print(f"gpu encode {time.time() - t0:.1f} s: status {est.item()}, {elens.item()} bytes", flush=True)
    assert est.item() == 0
    got = enc[:elens.item()].cpu().numpy()
    count = int.from_bytes(got[:8].tobytes(), "little")
    print(f"adaptive symbols {count}, sha256 {hashlib.sha256(got.tobytes()).hexdigest()[:16]}", flush=True)
    back = torch.empty_like(raw)
    blens, bst = torch.zeros(1, **i64), torch.full((1,), -1, dtype=torch.int32, device=dev)
    t0 = time.time()
    work = hc.decompress_adapt_batch(enc, eoffs, elens, back, offs, lens, blens, bst)
    torch.cuda.synchronize()
    del work
    print(f"gpu decode {time.time() - t0:.1f} s: status {bst.item()}, {blens.item()} bytes", flush=True)
    assert bst.item() == 0 and blens.item() == N
    assert torch.equal(back, raw), "GPU round trip differs"
    print("gpu round trip exact", flush=True)
    del back
    host = raw.cpu().numpy()
    del raw
    torch.cuda.empty_cache()
    t0 = time.time()
    want_st, want = oracle_mod.compress(host, True, True, W)
    print(f"oracle encode {time.time() - t0:.1f} s: status {want_st}, {len(want)} bytes", flush=True)
    assert want_st == 0 and len(want) == len(got) and np.array_equal(np.frombuffer(want, np.uint8), got)
    print("gpu encoding byte-identical to the oracle's", flush=True)
