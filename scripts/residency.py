"""How many FGK waves share each SIMD during the bench workload (diagnostic).

Uses the kernels' trace hook (hc_debug_set_trace in hc_fgk.hip): every wave records its start
and end time (s_memtime, per XCD) and where it ran (HW_ID | XCC_ID << 16). Reports per kernel:
the time-weighted mean and the peak number of co-resident waves per SIMD, the mean wave life
and the span of the launch on XCD 0 (cycles), and how many "rounds" of waves a SIMD ran.

    python scripts/residency.py [--streams 8192] [--kind photo]
"""
import argparse
import collections
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "huffman-codec_amd", "python"))


def analyze(name, tr):
    n = tr.shape[0]
    ev = collections.defaultdict(list)
    life = 0.0
    for t0, t1, hw in tr.tolist():
        key = hw & ~0xF  # xcc, se, sh, cu, simd (not the wave slot)
        ev[key].append((t0, 1))
        ev[key].append((t1, -1))
        life += t1 - t0
    peaks, means, rounds = [], [], []
    for key, v in ev.items():
        v.sort(key=lambda e: (e[0], e[1]))
        cur = peak = 0
        area = 0.0
        last = v[0][0]
        for t, d in v:
            area += cur * (t - last)
            last = t
            cur += d
            peak = max(peak, cur)
        span = v[-1][0] - v[0][0]
        peaks.append(peak)
        means.append(area / span if span else 0)
        starts = sorted(t for t, d in v if d > 0)
        # a new round starts when a wave begins after some wave of this SIMD already ended
        ends = sorted(t for t, d in v if d < 0)
        rounds.append(1 + sum(1 for s in starts if s > ends[0]))
    # per SIMD: each wave's life relative to that SIMD's longest, by rank (shortest first)
    by = collections.defaultdict(list)
    for t0, t1, hw in tr.tolist():
        by[hw & ~0xF].append(t1 - t0)
    ranks = collections.defaultdict(list)
    for v in by.values():
        v.sort()
        for r, x in enumerate(v):
            ranks[r].append(x / v[-1])
    rel = " ".join(f"{sum(x) / len(x):.2f}" for _, x in sorted(ranks.items()))
    x0 = [r for r in tr.tolist() if (r[2] >> 16) == 0]
    span0 = max(r[1] for r in x0) - min(r[0] for r in x0) if x0 else 0
    print(f"{name}: {n} waves on {len(ev)} SIMDs; co-resident waves per SIMD: time-weighted mean "
          f"{sum(means) / len(means):.2f}, peak max {max(peaks)} / mean {sum(peaks) / len(peaks):.2f}; "
          f"waves started after another ended on the same SIMD: mean {sum(rounds) / len(rounds) - 1:.2f}; "
          f"mean wave life {life / n:.3g} cycles, launch span on XCD 0 {span0:.3g} cycles; wave life / the "
          f"SIMD's longest, by rank: {rel}", flush=True)
    # balance across SIMDs (s_memtime counts per XCD: compare within one): per SIMD, when its
    # first wave started and its last ended, relative to the XCD's first start, as fractions of
    # the XCD's span; and the spread of wave lives over the streams
    for xcc in sorted({r[2] >> 16 for r in tr.tolist()})[:2]:
        rows = [r for r in tr.tolist() if (r[2] >> 16) == xcc]
        t0 = min(r[0] for r in rows)
        span = max(r[1] for r in rows) - t0
        first = collections.defaultdict(lambda: float("inf"))
        last = collections.defaultdict(float)
        for a, b, hw in rows:
            first[hw & ~0xF] = min(first[hw & ~0xF], a)
            last[hw & ~0xF] = max(last[hw & ~0xF], b)
        def pct(v):
            v = sorted(v)
            return " ".join(f"{v[int(q * (len(v) - 1))]:.3f}" for q in (0, 0.1, 0.5, 0.9, 1))
        print(f"  XCD {xcc}: span {span:.3g}; SIMD first start / span (min p10 p50 p90 max): "
              f"{pct([(x - t0) / span for x in first.values()])}; SIMD last end / span: "
              f"{pct([(x - t0) / span for x in last.values()])}", flush=True)
    lives = sorted(b - a for a, b, _ in tr.tolist())
    m = sum(lives) / len(lives)
    print(f"  wave life / mean (min p10 p50 p90 max): " + " ".join(
        f"{lives[int(q * (len(lives) - 1))] / m:.3f}" for q in (0, 0.1, 0.5, 0.9, 1)), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=8192)
    ap.add_argument("--kind", default="photo")
    ap.add_argument("--no-diff", action="store_true")
    args = ap.parse_args()
    import torch
    import hcodec as hc
    L = hc.use_debug_build(True)  # hc_debug_set_trace: debug build only
    L.hc_debug_set_trace.argtypes = [ctypes.c_void_p]
    S, N = args.streams, 512 * 512
    dev = torch.device("cuda", 0)
    raw = torch.empty(S * N, dtype=torch.uint8, device=dev)
    hc.synth_batch(args.kind, 0, S, 512, 512, raw, N)
    offs = torch.arange(S, dtype=torch.int64, device=dev) * N
    lens = torch.full((S,), N, dtype=torch.int64, device=dev)
    cap = 2 * N + 4096
    enc = torch.empty(S * cap, dtype=torch.uint8, device=dev)
    eoffs = torch.arange(S, dtype=torch.int64, device=dev) * cap
    ecaps = torch.full((S,), cap, dtype=torch.int64, device=dev)
    elens = torch.zeros(S, dtype=torch.int64, device=dev)
    est = torch.zeros(S, dtype=torch.int32, device=dev)
    back = torch.empty_like(raw)
    blens = torch.zeros_like(lens)
    bst = torch.zeros_like(est)
    trace = torch.zeros(3 * S, dtype=torch.int64, device=dev)
    # warm run without the trace
    hc.compress_batch(raw, offs, lens, enc, eoffs, ecaps, elens, est, use_diff=not args.no_diff)
    torch.cuda.synchronize()
    assert L.hc_debug_set_trace(ctypes.c_void_p(trace.data_ptr())) == 0
    try:
        hc.compress_batch(raw, offs, lens, enc, eoffs, ecaps, elens, est, use_diff=not args.no_diff)
        torch.cuda.synchronize()
        analyze("encode_kernel", trace.view(S, 3).cpu().numpy())
        trace.zero_()
        hc.decompress_batch(enc, eoffs, elens, back, offs, lens, blens, bst)
        torch.cuda.synchronize()
        analyze("decode_kernel", trace.view(S, 3).cpu().numpy())
    finally:
        L.hc_debug_set_trace(ctypes.c_void_p(0))
        torch.cuda.synchronize()
    assert torch.equal(back, raw)


if __name__ == "__main__":
    main()
