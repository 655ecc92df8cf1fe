"""GPU check of the encoder's per-stream mode vote (hc_fgk.hip enc_mode_kernel) against a numpy
model of the same rule: run-start bytes of a 16 KB sample (the whole stream up to 16 KB, else
64 segments of 256 bytes spread evenly over it, each segment's first symbol starting a run),
diff model applied, the share of the 16 most frequent ones: the path cache at >= 60 %, or at
>= 9 % when the batch does not fit table mode's residency (low_occ 0); at most 4 distinct
run-start bytes: the small-alphabet kernel. The vote only picks which of three bit-identical
encoders runs (tests/test_gpu_tab.py checks both against the reference),
so this pins speed, not output: hd01 -c -m alone must take the level tables (its first 16 KB
alone voted for the cache: 108 ms against 55 ms).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CACHE, TABLES, SMALL = -0x7A1, -0x7A0, -0x7A2


def vote_model(m, diff, low_occ):
    m = np.frombuffer(bytes(m), np.uint8).astype(np.int64)
    n = len(m)
    spread = n > 16384
    nseg = 64 if spread else (n + 255) // 256
    h = np.zeros(256, np.int64)
    total = 0
    prev_sym = 0
    for k in range(nseg):
        o = (((n - 256) * k // 63) & ~3) if spread else 256 * k
        ln = min(n - o, 256)
        raw = m[o:o + ln]
        pr = m[o - 1] if o else 0  # the byte before the segment (m[-1] = 0)
        s = (raw - np.concatenate([[pr], raw[:-1]])) & 255 if diff else raw
        before = np.concatenate([[prev_sym], s[:-1]])
        start = s != before
        if spread or k == 0:
            start[0] = True
        np.add.at(h, s[start], 1)
        total += int(start.sum())
        prev_sym = int(s[-1])
    top = int(np.sort(h)[::-1][:16].sum())
    cache = total == 0 or 100 * top >= 60 * total or (100 * top >= 9 * total and not low_occ)
    if total and int((h != 0).sum()) <= 4:  # a small alphabet: the small-alphabet kernel
        return SMALL
    return CACHE if cache else TABLES


def _inputs(oracle_mod):
    out = []
    for kind in ("photo", "noise", "grad"):
        for k in range(2):
            out.append((f"{kind}{k}", oracle_mod.synth(kind, k).tobytes()))
    st, hd01 = oracle_mod.decompress(open(_corpus("hd01.cm.huf"), "rb").read())
    assert st == 0
    out.append(("hd01", hd01))
    rng = np.random.default_rng(7)
    photo = out[0][1]
    for n in (0, 1, 3, 255, 256, 257, 5000, 16383, 16384, 16385, 20001, 70003):
        out.append((f"photo[:{n}]", photo[:n] if n <= len(photo) else photo))
    # flat top, wide alphabet below: the case the prefix sample misjudged
    flat = bytes(20000) + rng.integers(0, 256, 200000, dtype=np.uint8).tobytes()
    out.append(("flat+noise", flat))
    out.append(("runs", np.repeat(rng.integers(0, 8, 3000, dtype=np.uint8), 37).tobytes()))
    return out


def _corpus(name):
    import os
    return os.path.join(os.path.dirname(__file__), "golden", "corpus", name)


@pytest.mark.parametrize("low_occ", [0, 1])
@pytest.mark.parametrize("diff", [False, True], ids=["c", "cm"])
def test_vote_matches_model(gpu, hc, oracle_mod, diff, low_occ):
    torch = gpu
    hc.use_debug_build(True)
    try:
        items = _inputs(oracle_mod)
        # odd offsets: the sample's dword loads must not depend on the stream's alignment
        offs, buf, at = [], bytearray(), 1
        for _, b in items:
            buf += bytes(at - len(buf))
            offs.append(at)
            buf += b
            at = len(buf) + 5
        buf += bytes(16)
        dev = torch.device("cuda", 0)
        inp = torch.tensor(np.frombuffer(bytes(buf), np.uint8), device=dev)
        o = torch.tensor(offs, dtype=torch.int64, device=dev)
        ln = torch.tensor([len(b) for _, b in items], dtype=torch.int64, device=dev)
        st = torch.zeros(len(items), dtype=torch.int32, device=dev)
        hc.debug_enc_votes(inp, o, ln, diff, low_occ, st)
        torch.cuda.synchronize()
        got = st.cpu().tolist()
        want = [vote_model(b, diff, low_occ) for _, b in items]
        bad = [(name, g, w) for (name, _), g, w in zip(items, got, want) if g != w]
        assert not bad, bad
        votes = dict(zip([name for name, _ in items], got))
        # the calibration points of the rule (hc_fgk.hip, above enc_mode_kernel)
        assert votes["noise0"] == TABLES
        if diff:
            assert votes["photo0"] == CACHE and votes["grad0"] == SMALL
            if low_occ:
                assert votes["hd01"] == TABLES
        assert votes["flat+noise"] == TABLES
    finally:
        hc.use_debug_build(False)
