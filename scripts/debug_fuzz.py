"""GPU debug aid: every fuzz case (tests/test_fuzz.py) whose GPU decode differs from the oracle."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in ('huffman-codec_amd/python', 'oracle', 'tests'):
    sys.path.insert(0, os.path.join(ROOT, d))
import torch  # noqa: F401
import hcodec as hc
import oracle as O
import test_fuzz as T

bad = 0
for name, data in T._mutants(O):
    st, want = O.decompress(data)
    st = T.ORACLE_CRASH.get(st, st)
    gst, got = hc.decompress(data)
    if gst != st or got != want:
        bad += 1
        k = next((j for j in range(min(len(got), len(want))) if got[j] != want[j]), min(len(got), len(want)))
        print(name, 'status', st, gst, 'len', len(want), len(got), 'first diff', k,
              'want', want[max(0, k - 4):k + 8].hex(), 'got', got[max(0, k - 4):k + 8].hex(),
              'count', int.from_bytes(data[:8], 'little'), 'flags', hex(data[8]) if len(data) > 8 else None)
print('bad', bad)
