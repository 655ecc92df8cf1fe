import sys, time, os
sys.path.insert(0, "huffman-codec_amd/python"); sys.path.insert(0, "oracle")
import torch, hcodec as hc, oracle, numpy as np
hc.use_debug_build(True)  # hc_debug_set_min_tree: debug build only
n = 1 << 26
pat = torch.tensor([1, 1, 2, 1, 1, 3, 1, 1, 2], dtype=torch.uint8, device="cuda")
raw = pat.repeat(n // pat.numel() + 1)[:n].contiguous()
cap = n // 2
enc = torch.zeros(cap, dtype=torch.uint8, device="cuda")
i64 = dict(dtype=torch.int64, device="cuda")
z = torch.zeros(1, **i64); elen = torch.zeros(1, **i64); est = torch.full((1,), -1, dtype=torch.int32, device="cuda")
for mt in (1, 2):
    hc.debug_set_min_tree(mt)
    torch.cuda.synchronize(); t0 = time.time()
    hc.compress_batch(raw, z, torch.tensor([n], **i64), enc, z, torch.tensor([cap], **i64), elen, est)
    torch.cuda.synchronize(); t1 = time.time()
    back = torch.zeros_like(raw); blen = torch.zeros(1, **i64); bst = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    hc.decompress_batch(enc, z, elen, back, z, torch.tensor([n], **i64), blen, bst)
    torch.cuda.synchronize(); t2 = time.time()
    print("tree", mt, "enc s", round(t1 - t0, 2), "dec s", round(t2 - t1, 2), "ns/sym", round((t1-t0)/n*1e9, 1), round((t2-t1)/n*1e9, 1), est.item(), bst.item(), torch.equal(back, raw), elen.item(), flush=True)
host = raw.cpu().numpy()
t0 = time.time(); st, want = oracle.compress(host, False, False, 512); t1 = time.time()
print("oracle enc s", round(t1 - t0, 2), "ns/sym", round((t1-t0)/n*1e9, 1), st, len(want) == elen.item(), os.cpu_count(), flush=True)
