"""GPU debug aid: batch-encode small inputs, report the first byte where the GPU differs from the oracle."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in ('huffman-codec_amd/python', 'oracle', 'tests'):
    sys.path.insert(0, os.path.join(ROOT, d))
import torch
import hcodec as hc
import oracle as O
from gpu_batch import compress_batch

raws = [b'a', b'ab', b'abc', b'abcdefgh', bytes(range(256)), bytes(range(256)) * 2, b'x' * 10,
        O.synth('grad', 0, 64, 64).tobytes(), O.synth('photo', 0, 64, 64).tobytes(),
        O.synth('grad', 0).tobytes()]
for diff in (False, True):
    st, encs, lens = compress_batch(hc, torch, raws, use_diff=diff)
    for i, (r, e) in enumerate(zip(raws, encs)):
        s, want = O.compress(r, diff, False, 512)
        if e == want:
            print(diff, i, len(r), 'match', len(e))
            continue
        k = next((j for j in range(min(len(e), len(want))) if e[j] != want[j]), min(len(e), len(want)))
        print(diff, i, len(r), 'DIFF at', k, 'len', len(e), len(want), 'st', st[i])
        print('   got ', e[max(0, k - 8):k + 16].hex())
        print('   want', want[max(0, k - 8):k + 16].hex())
