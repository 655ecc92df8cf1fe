"""Error-path parity under malformed input: truncated, bit-flipped and forged
streams of all four modes, decoded by

  * the reference binary itself vs the oracle (CPU, when oracle/_ref is built): pins the oracle's
    exit codes and outputs on malformed data (main.cpp:99-104, transform.cpp:170-184, 354-358,
    394-398, headers.cpp:67-98);
  * the GPU (single-buffer API for every mode, batch API for the non-adaptive ones) vs the
    oracle: same status, same bytes.

Inputs the reference crashes on (a forged block size 0 divides by zero, transform.cpp:415; a
forged W*H beyond memory throws bad_alloc) have documented codes of their own here
(HC_ERR_BLOCK_SIZE / HC_ERR_TOO_LARGE); the CPU test checks that the oracle gives one of those
(100 / 101 in its own numbering) exactly when the reference dies by a signal. Mutations are
seeded: the same cases every run.
"""
import random

import pytest

MODES = {"c": (False, False), "cm": (True, False), "ca": (False, True), "cma": (True, True)}
ORACLE_CRASH = {100: 66, 101: 67}  # oracle code -> C ABI code (HC_ERR_BLOCK_SIZE, HC_ERR_TOO_LARGE)


def _bases(oracle_mod):
    out = []
    for kind, w, h in (("photo", 64, 48), ("grad", 40, 32), ("noise", 16, 16)):
        raw = oracle_mod.synth(kind, 7, w, h).tobytes()
        for m, (d, a) in MODES.items():
            st, enc = oracle_mod.compress(raw, d, a, w)
            assert st == 0
            out.append((f"{kind}.{m}", enc))
    return out


def _mutants(oracle_mod, seed=2024, per_base=40):
    rng = random.Random(seed)
    cases = []
    for name, enc in _bases(oracle_mod):
        n = len(enc)
        muts = [("trunc0", b""), ("trunc8", enc[:8]), ("trunc9", enc[:9]), ("trunc-1", enc[:-1]),
                ("flags^40", enc[:8] + bytes([enc[8] ^ 0x40]) + enc[9:]),
                ("flags^80", enc[:8] + bytes([enc[8] ^ 0x80]) + enc[9:]),
                ("count+1", (int.from_bytes(enc[:8], "little") + 1).to_bytes(8, "little") + enc[8:]),
                ("count-1", (max(0, int.from_bytes(enc[:8], "little") - 1)).to_bytes(8, "little") + enc[8:]),
                ("count*2", (int.from_bytes(enc[:8], "little") * 2).to_bytes(8, "little") + enc[8:]),
                ("count=2^40", (1 << 40).to_bytes(8, "little") + enc[8:])]
        for k in range(per_base - len(muts)):
            b = bytearray(enc)
            r = rng.random()
            if r < 0.4 and n > 9:  # one payload bit
                p = rng.randrange(9, n)
                b[p] ^= 1 << rng.randrange(8)
                tag = f"bit@{p}"
            elif r < 0.6 and n > 10:  # truncate inside the payload
                p = rng.randrange(10, n)
                b = b[:p]
                tag = f"cut@{p}"
            elif r < 0.8 and n > 9:  # a random byte
                p = rng.randrange(9, n)
                b[p] = rng.randrange(256)
                tag = f"byte@{p}"
            else:  # a few bits of the count
                b[rng.randrange(0, 3)] ^= 1 << rng.randrange(8)
                tag = "countbit"
            muts.append((tag, bytes(b)))
        cases += [(f"{name}:{t}", m) for t, m in muts]
    return cases


def test_fuzz_oracle_vs_reference(oracle_mod, tmp_path):
    if not oracle_mod.ref_available():
        pytest.skip("reference binary not built (oracle/_ref)")
    for name, data in _mutants(oracle_mod):
        rc, out, _ = oracle_mod.run_ref(["-d"], data, str(tmp_path), o2=oracle_mod.ref_available(o2=True),
                                        timeout=120)
        st, mine = oracle_mod.decompress(data)
        if rc < 0:  # the reference died by a signal: a documented divergence code here
            assert st in ORACLE_CRASH, (name, rc, st)
            continue
        assert st not in ORACLE_CRASH, (name, rc, st)
        assert st == rc, (name, rc, st)
        if rc == 0:
            assert mine == out, name


@pytest.mark.gpu
def test_fuzz_gpu_vs_oracle(gpu, hc, oracle_mod):
    cases = _mutants(oracle_mod)
    batchable = []
    for name, data in cases:
        st, want = oracle_mod.decompress(data)
        st = ORACLE_CRASH.get(st, st)
        got_st, got = hc.decompress(data)
        assert got_st == st, (name, st, got_st)
        assert got == want, name
        if len(data) < 9 or not (data[8] & 0x40):
            batchable.append((name, data, st, want))
    # the same non-adaptive streams through the host batch API (device batch kernels)
    sts, outs, _ = hc.decompress_host_batch([d for _, d, _, _ in batchable],
                                            [max(len(w), 1) + 64 for _, _, _, w in batchable])
    for (name, _, st, want), got_st, got in zip(batchable, sts, outs):
        assert got_st == st, (name, st, got_st)
        assert got == want, name
