"""`huffman-codec` CLI contract (src/main.cpp:152-221) against the reference binary.

CPU-side: option parsing, help text, exit codes 1-6 and 12 decided before device work.
GPU-side (marked): full compress / decompress through the CLI, byte-identical files.
"""
import os
import subprocess

import pytest

from conftest import ROOT

REF = os.path.join(ROOT, "oracle", "_ref", "huffman-codec")


@pytest.fixture(scope="module")
def cli(hc):
    if not os.path.exists(hc.CLI_PATH):
        subprocess.run(["make", "-s", "-C", hc.PKG], check=True)
    return hc.CLI_PATH


def run(binary, args, cwd):
    r = subprocess.run([binary] + args, capture_output=True, cwd=cwd)
    return r.returncode, r.stdout, r.stderr


CASES = [
    ["-h"],
    ["-c", "-h", "-q"],
    ["-q"],
    ["-i"],
    ["-c"],
    ["-m", "-a"],
    ["-w", "0", "-i", "in.bin"],
    ["-d", "-w", "0", "-i", "missing.bin"],
    ["-i", "missing.bin"],
    ["-a", "-w", "7", "-i", "in.bin"],
    ["-a", "-w", "100", "-i", "in.bin"],
    ["-c", "-m", "-a", "-w", "3", "-i", "in.bin"],
]


@pytest.mark.skipif(not os.path.exists(REF), reason="reference binary not built")
@pytest.mark.parametrize("args", CASES, ids=[" ".join(c) for c in CASES])
def test_cli_pre_device_paths_match_reference(cli, tmp_path, args):
    (tmp_path / "in.bin").write_bytes(bytes(range(256)) * 3 + bytes(3))  # 771 bytes
    want = run(REF, args, tmp_path)
    got = run(cli, args, tmp_path)
    assert got[0] == want[0]
    assert got[1] == want[1]
    if want[0] != 0:
        assert got[2] == want[2]


def test_cli_help_text(cli, tmp_path):
    rc, out, _ = run(cli, ["-h"], tmp_path)
    assert rc == 0 and out.startswith(b"USAGE:\n  huffman-codec [-cm] -i IFILE [-o OFILE]\n")


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(REF), reason="reference binary not shipped")
def test_cli_roundtrip_matches_reference(cli, gpu, oracle_mod, tmp_path):
    raw = oracle_mod.synth("photo", 5, 128, 96).tobytes()
    (tmp_path / "in.raw").write_bytes(raw)
    for args in (["-c"], ["-c", "-m"], ["-c", "-a", "-w", "128"], ["-m", "-a", "-w", "128"]):
        r1 = run(REF, args + ["-i", "in.raw", "-o", "ref.huf"], tmp_path)
        r2 = run(cli, args + ["-i", "in.raw", "-o", "gpu.huf"], tmp_path)
        assert r1[0] == r2[0] == 0 and r1[2] == r2[2].replace(b"gpu.huf", b"ref.huf")
        assert (tmp_path / "ref.huf").read_bytes() == (tmp_path / "gpu.huf").read_bytes(), args
        r3 = run(cli, ["-d", "-i", "gpu.huf", "-o", "back.raw"], tmp_path)
        assert r3[0] == 0 and (tmp_path / "back.raw").read_bytes() == raw


@pytest.mark.gpu
def test_cli_decode_errors_match_reference_codes(cli, gpu, vectors, tmp_path):
    for v in vectors["decompress"]:
        (tmp_path / "bad.huf").write_bytes(bytes.fromhex(v["input"]))
        rc, _, _ = run(cli, ["-d", "-i", "bad.huf", "-o", "o.bin"], tmp_path)
        assert rc == v["rc"], v["name"]
