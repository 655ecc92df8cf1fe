"""Every BASELINE.json config, measured in one run on one MI355X (bench.py reports only the
N=1 line of the headline metric; this is the table behind DESIGN.md §4).

  C1  data/hd01.raw `-c -m` on the CPU reference binary (oracle/_ref, Makefile flags) — the
      input is rebuilt from the committed reference output tests/golden/corpus/hd01.cm.huf
      by the reference binary itself (`-d`), since /root/reference is not on the GPU box
  C2  one synthetic 512x512 photo stream `-c -m` (one wavefront: latency of a lone stream)
  C3  4096 photo streams `-c`
  C4  `-c -a -w 4096` on one 4096x4096 photo matrix (and `-c -a -m`), single-buffer API
  C5  the per-GPU shard of the 8-GPU batch: 8192 photo streams `-c -m` round trip (= bench.py)

GPU times are HIP events around the device work (inputs resident in HBM), except C4, which
goes through the host single-buffer API (H2D + kernels + D2H, wall clock). Every result is
checked (round trip exact; C1-C4 byte-compared with the oracle where the size allows).

    python scripts/bench_configs.py [--out profiles/r01_configs.json]
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "huffman-codec_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
N = 512 * 512


def batch_round_trip(hc, torch, S, kind, use_diff, reps=3):
    dev = torch.device("cuda", 0)
    raw = torch.empty(S * N, dtype=torch.uint8, device=dev)
    hc.synth_batch(kind, 0, S, 512, 512, raw, N)
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
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    best = None
    for _ in range(reps + 1):  # the first is warm-up
        ev[0].record()
        hc.compress_batch(raw, offs, lens, enc, eoffs, ecaps, elens, est, use_diff=use_diff)
        ev[1].record()
        hc.decompress_batch(enc, eoffs, elens, back, offs, lens, blens, bst)
        ev[2].record()
        torch.cuda.synchronize()
        t = (ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2]))
        best = t if best is None or sum(t) < sum(best) else best
    ok = bool((est == 0).all() and (bst == 0).all() and torch.equal(back, raw))
    first = enc[: int(elens[0])].cpu().numpy().tobytes()
    return best, ok, int(elens.sum()), first, raw[:N].cpu().numpy().tobytes()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--skip-c4", action="store_true")
    ap.add_argument("--only", default="C1,C2,C3,C4,C5", help="comma-separated subset of C1..C5")
    args = ap.parse_args()
    only = set(args.only.upper().split(","))
    if args.skip_c4:
        only.discard("C4")
    import torch
    import hcodec as hc
    import oracle
    res = {"device": hc.device_info()}

    # C1: the reference binary on hd01 (rebuilt from the committed reference output)
    if "C1" in only and oracle.ref_available():
        with tempfile.TemporaryDirectory() as d:
            huf = os.path.join(ROOT, "tests", "golden", "corpus", "hd01.cm.huf")
            subprocess.run([oracle.REF_BIN, "-d", "-i", huf, "-o", os.path.join(d, "hd01.raw")], check=True,
                           capture_output=True)
            t0 = time.perf_counter()
            subprocess.run([oracle.REF_BIN, "-c", "-m", "-i", os.path.join(d, "hd01.raw"), "-o",
                            os.path.join(d, "o.huf")], check=True, capture_output=True)
            t1 = time.perf_counter()
            out = open(os.path.join(d, "o.huf"), "rb").read()
            raw = open(os.path.join(d, "hd01.raw"), "rb").read()
            st, gpu_out = hc.compress(raw, True, False, 512)
            res["C1"] = {"what": "hd01.raw -c -m, reference binary (-O0), 1 core", "seconds": round(t1 - t0, 4),
                         "bytes": len(out), "sha256_16": hashlib.sha256(out).hexdigest()[:16],
                         "gpu_single_api_identical": st == 0 and gpu_out == out}
    print(json.dumps({"C1": res.get("C1")}), flush=True)

    # C2: one stream (a lone wavefront)
    if "C2" in only:
        (te, td), ok, nbytes, first, raw0 = batch_round_trip(hc, torch, 1, "photo", True, reps=5)
        res["C2"] = {"what": "1 x 512x512 photo -c -m, one wavefront", "encode_ms": round(te, 3),
                     "decode_ms": round(td, 3), "bytes": nbytes, "round_trip_exact": ok,
                     "oracle_identical": first == oracle.compress(raw0, True, False, 512)[1]}
        print(json.dumps({"C2": res["C2"]}), flush=True)

    # C3: 4096 streams -c
    if "C3" in only:
        (te, td), ok, nbytes, first, raw0 = batch_round_trip(hc, torch, 4096, "photo", False)
        res["C3"] = {"what": "4096 x 512x512 photo -c", "encode_ms": round(te, 3), "decode_ms": round(td, 3),
                     "GiBps_enc_dec": round(4096 * N / ((te + td) * 1e-3) / 2**30, 4), "bytes": nbytes,
                     "round_trip_exact": ok, "stream0_oracle_identical": first == oracle.compress(raw0, False, False, 512)[1]}
        print(json.dumps({"C3": res["C3"]}), flush=True)

    # C4: one 4096x4096 matrix, adaptive block RLE, single-buffer API (host buffers)
    if "C4" in only:
        buf = torch.empty(4096 * 4096, dtype=torch.uint8, device="cuda")
        hc.synth_batch("photo", 0, 1, 4096, 4096, buf, 0)
        raw = buf.cpu().numpy().tobytes()
        for mode, use_diff in (("-c -a", False), ("-c -a -m", True)):
            t0 = time.perf_counter()
            st, out = hc.compress(raw, use_diff, True, 4096)
            t1 = time.perf_counter()
            st2, back = hc.decompress(out)
            t2 = time.perf_counter()
            res["C4" + ("m" if use_diff else "")] = {
                "what": f"4096x4096 photo {mode} -w 4096, single-buffer API incl. PCIe", "encode_s": round(t1 - t0, 3),
                "decode_s": round(t2 - t1, 3), "bytes": len(out), "sha256_16": hashlib.sha256(out).hexdigest()[:16],
                "round_trip_exact": st == 0 and st2 == 0 and back == raw}
            print(json.dumps({"C4" + ("m" if use_diff else ""): res["C4" + ("m" if use_diff else "")]}), flush=True)

    # C5: the per-GPU shard (bench.py's workload)
    if "C5" in only:
        (te, td), ok, nbytes, _, _ = batch_round_trip(hc, torch, 8192, "photo", True)
        res["C5"] = {"what": "8192 x 512x512 photo -c -m round trip (per-GPU shard of 65536)", "encode_ms": round(te, 3),
                     "decode_ms": round(td, 3), "GiBps_enc_dec": round(8192 * N / ((te + td) * 1e-3) / 2**30, 4),
                     "bytes": nbytes, "round_trip_exact": ok}
        print(json.dumps({"C5": res["C5"]}), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
