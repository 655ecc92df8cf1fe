"""The encoder's second stream (hc_compress_batch_aux, include/hcodec.h): the path-cache and the
table-mode launches of a batch mixing skewed (photo -c -m: cache) and flat (noise: tables)
alphabets give the same bytes whether the table launches run on the caller's stream
(aux NULL, the C hc_compress_batch), on the module's side stream ("auto") or on a stream the
caller passes, and under HIP graph capture (fork / join by events inside the capture), all
equal to the oracle (the reference's algorithm: transform.cpp:363-384)."""
import pytest

from gpu_batch import pack, unpack

pytestmark = pytest.mark.gpu

W = H = 96


def mixed(oracle_mod):
    kinds = ["photo", "noise", "photo", "grad", "noise", "photo", "noise", "photo"]
    return [oracle_mod.synth(k, i, W, H).tobytes() for i, k in enumerate(kinds)]


def buffers(hc, torch, raws):
    din, ioffs, ilens, _ = pack(torch, raws)
    caps = [hc.compress_bound(len(r)) for r in raws]
    dout, ooffs, _, ocaps = pack(torch, [b""] * len(raws), caps)
    olens = torch.zeros(len(raws), dtype=torch.int64, device="cuda")
    st = torch.full((len(raws),), -1, dtype=torch.int32, device="cuda")
    return din, ioffs, ilens, dout, ooffs, ocaps, olens, st


@pytest.mark.parametrize("aux", ["none", "auto", "caller"])
def test_aux_stream_variants(gpu, hc, oracle_mod, aux):
    torch = gpu
    raws = mixed(oracle_mod)
    din, ioffs, ilens, dout, ooffs, ocaps, olens, st = buffers(hc, torch, raws)
    stream = torch.cuda.Stream()
    side = {"none": None, "auto": "auto", "caller": torch.cuda.Stream()}[aux]
    hc.compress_batch(din, ioffs, ilens, dout, ooffs, ocaps, olens, st, use_diff=True, stream=stream,
                      aux_stream=side)
    stream.synchronize()
    assert st.cpu().tolist() == [0] * len(raws)
    got = unpack(torch, dout, ooffs, olens)
    for r, g in zip(raws, got):
        want = oracle_mod.compress(r, True, False, 512)
        assert want[0] == 0 and g == want[1]


def test_aux_stream_graph_capture(gpu, hc, oracle_mod):
    """compress (cache + table launches forked onto a caller stream) and decompress captured in
    one graph, replayed twice on fresh inputs: the bytes of each replay equal the oracle's"""
    torch = gpu
    raws = mixed(oracle_mod)
    din, ioffs, ilens, dout, ooffs, ocaps, olens, st = buffers(hc, torch, raws)
    back = torch.zeros_like(din)
    blens = torch.zeros_like(ilens)
    bst = torch.full_like(st, -1)
    side = torch.cuda.Stream()
    # warm up outside the capture (library init, lazy module loads)
    hc.compress_batch(din, ioffs, ilens, dout, ooffs, ocaps, olens, st, use_diff=True, aux_stream=side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cap = torch.cuda.current_stream()
        hc.compress_batch(din, ioffs, ilens, dout, ooffs, ocaps, olens, st, use_diff=True, stream=cap,
                          aux_stream=side)
        hc.decompress_batch(dout, ooffs, olens, back, ioffs, ilens, blens, bst, stream=cap)
    for rep in range(2):
        fresh = [oracle_mod.synth(k, 10 * rep + i, W, H).tobytes()
                 for i, k in enumerate(["noise", "photo", "photo", "noise", "grad", "photo", "noise", "photo"])]
        d2, _, _, _ = pack(torch, fresh)
        din.copy_(d2)
        st.fill_(-1)
        bst.fill_(-1)
        back.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert st.cpu().tolist() == [0] * len(fresh) and bst.cpu().tolist() == [0] * len(fresh)
        got = unpack(torch, dout, ooffs, olens)
        for r, e in zip(fresh, got):
            want = oracle_mod.compress(r, True, False, 512)
            assert e == want[1]
        assert unpack(torch, back, ioffs, blens) == fresh
