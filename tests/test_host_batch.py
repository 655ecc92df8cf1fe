"""Host-buffer batches (hc_compress_host_batch / hc_compress_adapt_host_batch /
hc_decompress_host_batch, csrc/hc_pipe.hip) and the `huffman-codec-batch` tool: byte-identical to
the oracle (the reference's algorithm) per stream, through the pipelined sub-batches, adaptive
(-a) matrices included. SURVEY.md §8f-1."""
import os
import subprocess

import pytest


def _inputs(oracle_mod):
    raws = [b"", b"\x01", b"abcabcabc", bytes(range(256)) * 3, b"\x07" * 1000]
    raws += [oracle_mod.synth(kind, k, 96, 64).tobytes() for kind in ("photo", "grad", "noise") for k in (0, 1)]
    raws += [oracle_mod.synth("photo", 5).tobytes(), bytes(1 << 20)]  # 512x512, 1 MiB of zeros
    return raws


@pytest.mark.gpu
@pytest.mark.parametrize("use_diff", [False, True])
@pytest.mark.parametrize("slots", ["default", "tiny"])
def test_host_batch_roundtrip_vs_oracle(gpu, hc, oracle_mod, use_diff, slots, monkeypatch):
    if slots == "tiny":  # three streams per sub-batch: both slots alternate several times
        monkeypatch.setenv("HC_PIPE_STREAMS", "3")
        monkeypatch.setenv("HC_PIPE_BYTES", "70000")
    raws = _inputs(oracle_mod)
    st, enc, _ = hc.compress_host_batch(raws, use_diff=use_diff)
    assert st == [0] * len(raws)
    for r, e in zip(raws, enc):
        s, want = oracle_mod.compress(r, use_diff, False, 512)
        assert s == 0 and e == want
    # decode with generous caps; the 1 MiB zero stream outgrows the device guess (8x its
    # encoded size) and is redone with the size it reports
    st, dec, _ = hc.decompress_host_batch(enc, [len(r) + 64 for r in raws])
    assert st == [0] * len(raws) and dec == raws


@pytest.mark.gpu
def test_host_batch_concurrent_calls(gpu, hc, oracle_mod):
    """calls from several host threads at once (ctypes drops the GIL): one takes the persistent
    pipeline slots, the others their own; every result byte-identical to the oracle, and a
    second round reuses the slots"""
    import threading
    sets = [[oracle_mod.synth(kind, k, 128, 96).tobytes() for k in range(6)] for kind in ("photo", "grad", "noise")]
    want = [[oracle_mod.compress(r, True, False, 512)[1] for r in raws] for raws in sets]
    for _ in range(2):
        got, errs = [None] * len(sets), []

        def work(i):
            try:
                st, enc, _ = hc.compress_host_batch(sets[i], use_diff=True)
                dst, dec, _ = hc.decompress_host_batch(enc, [len(r) for r in sets[i]])
                got[i] = (st, enc, dst, dec)
            except Exception as e:  # surfaced below
                errs.append(e)

        th = [threading.Thread(target=work, args=(i,)) for i in range(len(sets))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs, errs
        for i, (st, enc, dst, dec) in enumerate(got):
            assert st == [0] * len(sets[i]) and enc == want[i]
            assert dst == [0] * len(sets[i]) and dec == sets[i]


@pytest.mark.gpu
def test_host_batch_statuses(gpu, hc, oracle_mod):
    raw = oracle_mod.synth("photo", 2, 64, 64).tobytes()
    _, want = oracle_mod.compress(raw, True, False, 512)
    adaptive = oracle_mod.compress(oracle_mod.synth("photo", 2, 64, 64).tobytes(), False, True, 64)[1]
    blobs = [want, want[:5], want[:len(want) // 2], adaptive, want]
    caps = [len(raw), 64, len(raw), 1 << 16, 10]
    st, dec, lens = hc.decompress_host_batch(blobs, caps)
    ref = [oracle_mod.decompress(b)[0] for b in blobs[:3]]
    assert st[0] == 0 and dec[0] == raw
    assert st[1] == ref[1] == hc.HC_ERR_HEADER
    assert st[2] == ref[2] == hc.HC_ERR_HUFFMAN
    assert st[3] == 0 and dec[3] == raw  # adaptive: through the batched adaptive path
    assert st[4] == hc.HC_ERR_CAPACITY and lens[4] == len(raw)  # too small: the size it needs
    # compress: a capacity below the result reports the needed length
    st, _, lens = hc.compress_host_batch([raw], use_diff=True, caps=[16])
    assert st == [hc.HC_ERR_CAPACITY] and lens == [len(want)]


@pytest.mark.gpu
def test_batch_cli_matches_oracle(gpu, hc, oracle_mod, tmp_path):
    raws = [oracle_mod.synth("photo", k, 128, 96).tobytes() for k in range(5)] + [b"", b"zz"]
    files = []
    for i, r in enumerate(raws):
        f = tmp_path / f"f{i}.raw"
        f.write_bytes(r)
        files.append(str(f))
    out_dir = tmp_path / "enc"
    out_dir.mkdir()
    p = subprocess.run([hc.BATCH_CLI_PATH, "-c", "-m", "-o", str(out_dir)] + files, capture_output=True, text=True)
    assert p.returncode == 0, p.stderr
    for f, r in zip(files, raws):
        got = (out_dir / (os.path.basename(f) + ".huf")).read_bytes()
        assert got == oracle_mod.compress(r, True, False, 512)[1]
    encs = sorted(str(x) for x in out_dir.iterdir())
    p = subprocess.run([hc.BATCH_CLI_PATH, "-d"] + encs, capture_output=True, text=True)
    assert p.returncode == 0, p.stderr
    for f, r in zip(files, raws):
        assert (out_dir / os.path.basename(f)).read_bytes() == r
    # a missing file: the reference's message and status, the others still coded
    p = subprocess.run([hc.BATCH_CLI_PATH, "-c", files[0], str(tmp_path / "nope")], capture_output=True, text=True)
    assert p.returncode == 5 and "given input file does not exist" in p.stderr
    assert (tmp_path / "f0.raw.huf").read_bytes() == oracle_mod.compress(raws[0], False, False, 512)[1]


@pytest.mark.gpu
@pytest.mark.parametrize("slots", ["default", "tiny"])
@pytest.mark.parametrize("use_diff", [False, True])
def test_adapt_host_batch_vs_oracle(gpu, hc, oracle_mod, use_diff, slots, monkeypatch):
    """-a matrices of several widths (and the reference's failures: width 0 -> 4, a size not a
    multiple of the width -> 6, a side below 8 -> 12) through hc_compress_adapt_host_batch, then
    decoded together with plain streams by hc_decompress_host_batch"""
    if slots == "tiny":
        monkeypatch.setenv("HC_PIPE_STREAMS", "2")
        monkeypatch.setenv("HC_PIPE_BYTES", "40000")
    mats = [(oracle_mod.synth("photo", k, w, h).tobytes(), w) for k, (w, h) in
            enumerate([(64, 64), (100, 37), (512, 512), (8, 8), (200, 129)])]
    mats += [(oracle_mod.synth("grad", 1, 96, 64).tobytes(), 96), (oracle_mod.synth("noise", 2, 40, 40).tobytes(), 40)]
    mats += [(b"x" * 640, 0), (b"y" * 650, 64), (b"z" * 640, 128)]  # statuses 4, 6, 12
    raws, widths = [m[0] for m in mats], [m[1] for m in mats]
    st, enc, _ = hc.compress_adapt_host_batch(raws, widths, use_diff=use_diff)
    for r, w, s, e in zip(raws, widths, st, enc):
        ws, want = oracle_mod.compress(r, use_diff, True, w) if w else (hc.HC_ERR_WIDTH, b"")
        assert s == ws and (s != 0 or e == want), (len(r), w)
    ok = [i for i, s in enumerate(st) if s == 0]
    plain = [oracle_mod.compress(raws[0], True, False, 512)[1]]
    blobs = [enc[i] for i in ok] + plain
    dst, dec, _ = hc.decompress_host_batch(blobs, [len(raws[i]) + 16 for i in ok] + [len(raws[0])])
    assert dst == [0] * len(blobs) and dec == [raws[i] for i in ok] + [raws[0]]


@pytest.mark.gpu
def test_batch_cli_adaptive(gpu, hc, oracle_mod, tmp_path):
    raws = [oracle_mod.synth("photo", k, 64, 48).tobytes() for k in range(4)]
    files = []
    for k, raw in enumerate(raws):
        f = tmp_path / f"m{k}.raw"
        f.write_bytes(raw)
        files.append(str(f))
    p = subprocess.run([hc.BATCH_CLI_PATH, "-c", "-a", "-m", "-w", "64"] + files, capture_output=True, text=True)
    assert p.returncode == 0, p.stderr
    for f, raw in zip(files, raws):
        assert open(f + ".huf", "rb").read() == oracle_mod.compress(raw, True, True, 64)[1]
    p = subprocess.run([hc.BATCH_CLI_PATH, "-d"] + [f + ".huf" for f in files], capture_output=True, text=True)
    assert p.returncode == 0, p.stderr
    for f, raw in zip(files, raws):
        assert open(f, "rb").read() == raw


def test_batch_cli_arguments(hc):
    """Argument handling decided before any device work (runs without a GPU)."""
    if not os.path.exists(hc.BATCH_CLI_PATH):
        subprocess.run(["make", "-s", "-C", hc.PKG], check=True)
    p = subprocess.run([hc.BATCH_CLI_PATH, "-h"], capture_output=True, text=True)
    assert p.returncode == 0 and p.stdout.startswith("USAGE:")
    assert subprocess.run([hc.BATCH_CLI_PATH], capture_output=True).returncode == 3
    assert subprocess.run([hc.BATCH_CLI_PATH, "-x", "f"], capture_output=True).returncode == 2
    assert subprocess.run([hc.BATCH_CLI_PATH, "-o"], capture_output=True).returncode == 1
    assert subprocess.run([hc.BATCH_CLI_PATH, "-w", "0", "f"], capture_output=True).returncode == 4
