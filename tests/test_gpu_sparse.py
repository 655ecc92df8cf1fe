"""GPU parity of the encoder's 2 KB sparse blocks (hc_fgk.hip rle_block, HC_SPARSE_KB = 2, the
shipping build; model: tests/rle_chunk_model.py rle_blocked): run-heavy streams that switch between
256-byte chunks and 2 KB blocks (sparse stretches, dense stretches, runs across the 258-byte cut and
the block edges) and grad photos, coded in both encoder modes and in both diff settings, byte for
byte against the oracle (transform.cpp:220-292 + 363-384), then decoded back.

Block edges: a stream whose first chunk has its run starts in at most two lanes switches to 2 KB
blocks after that chunk, so its blocks start at byte 256 + 2048 k. `_edge_streams` puts a run
start at every distance 0..258 before the edge 256 + 2 * 2048 (so the run counter R carried into
that block takes every phase of the 258-byte cut) and ends the run 0..6 bytes around the next edge.
The 1 KB variant (HC_SPARSE_KB = 1, not shipped) is pinned by test_rle_model's block = 1024 case only."""
import numpy as np
import pytest

from gpu_batch import compress_batch, decompress_batch
from test_rle_model import _run_heavy

pytestmark = pytest.mark.gpu


def _streams(oracle_mod):
    rng = np.random.default_rng(17)
    raws = [_run_heavy(rng, int(rng.integers(4000, 70000))) for _ in range(40)]
    # pure runs at every phase of the 258-byte cut against the block edges
    for k in range(12):
        raws.append(bytes([7]) * (1024 * 9 + 37 * k) + bytes([9]) * (300 + 211 * k) + bytes([7]) * 5000)
    raws += [oracle_mod.synth("grad", k, 512, 64 + 8 * k).tobytes() for k in range(4)]
    return raws + _edge_streams()


def _edge_streams(edge=256 + 2 * 2048, block=2048):
    """a run of 9s starting r bytes before a 2 KB block edge (r = 0..258: every carried counter
    phase at the edge, r = 258 the one right after a 258-byte cut), ending (r % 7) - 3 bytes
    around the next edge, inside runs of 7s"""
    raws = []
    for r in range(259):
        start = edge - r
        length = r + block + (r % 7) - 3
        raws.append(bytes([7]) * start + bytes([9]) * length + bytes([7]) * 3000)
    return raws


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("use_diff", [True, False])
def test_sparse_blocks_vs_oracle(gpu, hc, oracle_mod, use_diff, mode):
    torch = gpu
    raws = _streams(oracle_mod)
    if use_diff:  # streams whose diff holds the runs
        raws = [np.cumsum(np.frombuffer(r, dtype=np.uint8), dtype=np.uint64).astype(np.uint8).tobytes()
                if i % 2 == 0 else r for i, r in enumerate(raws)]
    hc.use_debug_build(True)
    try:
        hc.debug_set_enc_tab(mode)  # 1: path cache, 2: level tables
        st, encs, _ = compress_batch(hc, torch, raws, use_diff)
    finally:
        hc.debug_set_enc_tab(0)
        hc.use_debug_build(False)
    assert st == [0] * len(raws)
    for i, (r, e) in enumerate(zip(raws, encs)):
        want = oracle_mod.compress(r, use_diff, False, 512)
        assert want[0] == 0 and e == want[1], f"stream {i} ({len(r)} bytes)"
    st, back, _ = decompress_batch(hc, torch, encs, [len(r) for r in raws])
    assert st == [0] * len(raws) and back == raws
