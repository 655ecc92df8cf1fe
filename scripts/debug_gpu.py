import sys, os, hashlib
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'huffman-codec_amd', 'python')); sys.path.insert(0, os.path.join(ROOT, 'oracle')); sys.path.insert(0, os.path.join(ROOT, 'tests'))
order = sys.argv[1] if len(sys.argv) > 1 else 'lib-first'
if order == 'torch-first':
    import torch
import hcodec as hc
print('info', hc.device_info(), flush=True)
import torch
print('torch', torch.cuda.is_available(), torch.version.hip, flush=True)
print('info2', hc.device_info(), flush=True)
import oracle as O
from gpu_batch import compress_batch, decompress_batch
raws = [O.synth('photo', k, 64, 64).tobytes() for k in range(4)] + [b'', b'\x01', b'abcabcabc']
st, encs, lens = compress_batch(hc, torch, raws, use_diff=True)
print('status', st, 'lens', lens, flush=True)
for r, e in zip(raws, encs):
    s, want = O.compress(r, True, False, 512)
    print(len(r), 'match' if e == want else 'DIFF', len(e), len(want), e[:16].hex(), want[:16].hex())
st, back, bl = decompress_batch(hc, torch, encs, [len(r) for r in raws])
print('dec status', st, bl, [b == r for b, r in zip(back, raws)])
print('single', hc.compress(raws[0], True, False, 64)[0])
