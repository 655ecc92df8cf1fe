import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "huffman-codec_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")
REF_DATA = "/root/reference/data"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libhcodec.so's HIP kernels)")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    if not os.path.exists(oracle.LIB_PATH):
        oracle.build()
    return oracle


@pytest.fixture(scope="session")
def hc():
    """libhcodec.so, built in-tree if needed. Raises (never falls back) if it cannot load."""
    import hcodec
    if not os.path.exists(hcodec.LIB_PATH):
        subprocess.run(["make", "-s", "-C", hcodec.PKG], check=True)
    hcodec.lib()
    return hcodec


@pytest.fixture(scope="session")
def digests():
    with open(os.path.join(GOLDEN, "digests.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def vectors():
    with open(os.path.join(GOLDEN, "vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def gpu(hc):
    import torch
    assert torch.cuda.is_available(), "GPU test on a host without a GPU"
    assert hc.device_ok(), "libhcodec.so reports no usable gfx950 device"
    return torch
