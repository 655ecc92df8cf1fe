#!/usr/bin/env python3
"""bench.py — encode+decode GiB/s of the MI355X huffman-codec on batched 512x512 .raw streams.

Workload (BASELINE.json configs[4], weak-scaled): every GPU owns a shard of S = 8192 synthetic
512x512 photo streams (seed 0x5EED, stream k = rank*S + j, generated in
HBM), and one step is the reference's full round trip on that shard: `-c -m` encode
(diff -> MNP-5 RLE -> FGK -> header, one fused kernel) then decode (FGK -> RLE revert -> diff
revert, one fused kernel). value = raw bytes of all ranks / step time (max over ranks), in
GiB/s. Decoded output is checked against the input (bit-exact) after the timed region.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Streams are independent, so ranks share nothing on the data path (scaling "weak"); after the
timed region RCCL all-reduces the verification counters and all-gathers the encoded sizes.
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "huffman-codec_amd", "python"))

METRIC = "encode+decode GiB/s on batched 512×512 .raw, 1/2/4/8 GPUs; bit-exact check"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# what bounds the FGK kernels: VALU + SALU instruction issue per CU at their occupancy (8 waves
# per SIMD), measured by scripts/micro/issue.hip (independent VALU 1.77, VALU:SALU 1:1 1.73,
# SALU alone 0.95 instructions / cycle / CU)
ISSUE_PEAK = 1.75
CLOCK_HZ = 2.4e9
N_RAW = 512 * 512


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--streams", type=int, default=8192, help="streams per GPU")
    ap.add_argument("--kind", default="photo", choices=["photo", "grad", "noise"])
    ap.add_argument("--no-diff", action="store_true", help="-c instead of -c -m")
    ap.add_argument("--cpu-sample", type=int, default=0, help="streams for the CPU baseline (0 = auto)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic", default=None, help="JSON with PMC-derived HBM bytes per launch")
    ap.add_argument("--gather", action="store_true",
                    help="after timing, gather every rank's encoded payloads into rank 0")
    return ap.parse_args()


def cpu_baseline(args, cores):
    """The reference binary itself (oracle/_ref, Makefile flags) on a bounded sample of the
    same workload, one process per stream over `cores` host cores; falls back to the oracle's
    C restatement (kind "port") when the binary was not shipped."""
    import subprocess
    from concurrent.futures import ThreadPoolExecutor

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    sample = args.cpu_sample or 8 * cores
    kind = "reference" if oracle.ref_available() else "port"
    raws = [oracle.synth(args.kind, k).tobytes() for k in range(sample)]
    mode = ["-c"] if args.no_diff else ["-c", "-m"]
    tmp = tempfile.mkdtemp(dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    try:
        for i, r in enumerate(raws):
            with open(os.path.join(tmp, f"{i}.raw"), "wb") as f:
                f.write(r)

        def enc(i):
            if kind == "reference":
                subprocess.run([oracle.REF_BIN] + mode + ["-i", f"{i}.raw", "-o", f"{i}.huf"], cwd=tmp,
                               check=True, capture_output=True)
            else:
                st, out = oracle.compress(raws[i], not args.no_diff, False, 512)
                with open(os.path.join(tmp, f"{i}.huf"), "wb") as f:
                    f.write(out)

        def dec(i):
            if kind == "reference":
                subprocess.run([oracle.REF_BIN, "-d", "-i", f"{i}.huf", "-o", f"{i}.out"], cwd=tmp, check=True,
                               capture_output=True)
            else:
                with open(os.path.join(tmp, f"{i}.huf"), "rb") as f:
                    st, out = oracle.decompress(f.read())
                with open(os.path.join(tmp, f"{i}.out"), "wb") as f:
                    f.write(out)

        with ThreadPoolExecutor(cores) as ex:
            t0 = time.perf_counter()
            list(ex.map(enc, range(sample)))
            t1 = time.perf_counter()
            list(ex.map(dec, range(sample)))
            t2 = time.perf_counter()
        ok = all(open(os.path.join(tmp, f"{i}.out"), "rb").read() == raws[i] for i in range(sample))
    finally:
        for fn in os.listdir(tmp):
            os.remove(os.path.join(tmp, fn))
        os.rmdir(tmp)
    total = sample * N_RAW
    return {"value": total / (t2 - t0) / 2**30, "unit": "GiB/s", "cores": cores, "kind": kind,
            "sample": f"{sample} x 512x512 {args.kind} streams, {' '.join(mode)} then -d, one process per "
                      f"stream on {cores} host cores ({'oracle/_ref/huffman-codec, reference Makefile flags -O0' if kind == 'reference' else 'oracle C restatement'})",
            "encode_GiBps": total / (t1 - t0) / 2**30, "decode_GiBps": total / (t2 - t1) / 2**30,
            "seconds": t2 - t0, "bit_exact": ok}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import hcdist
    import hcodec as hc

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    if not hc.device_ok():
        raise SystemExit("libhcodec.so: no usable gfx950 device")

    S = args.streams
    use_diff = not args.no_diff
    cap = 2 * N_RAW + 4096
    raw = torch.empty(S * N_RAW, dtype=torch.uint8, device=dev)
    hc.synth_batch(args.kind, rank * S, S, 512, 512, raw, N_RAW)
    offs = torch.arange(S, dtype=torch.int64, device=dev) * N_RAW
    lens = torch.full((S,), N_RAW, dtype=torch.int64, device=dev)
    enc = torch.empty(S * cap, dtype=torch.uint8, device=dev)
    eoffs = torch.arange(S, dtype=torch.int64, device=dev) * cap
    ecaps = torch.full((S,), cap, dtype=torch.int64, device=dev)
    elens = torch.zeros(S, dtype=torch.int64, device=dev)
    est = torch.zeros(S, dtype=torch.int32, device=dev)
    back = torch.empty_like(raw)
    blens = torch.zeros_like(lens)
    bst = torch.zeros_like(est)
    stream = torch.cuda.current_stream(dev)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        hc.compress_batch(raw, offs, lens, enc, eoffs, ecaps, elens, est, use_diff=use_diff, stream=stream)
        if ev is not None:
            ev[1].record(stream)
        hc.decompress_batch(enc, eoffs, elens, back, offs, lens, blens, bst, stream=stream)
        if ev is not None:
            ev[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    enc_ms = sum(e[0].elapsed_time(e[1]) for e in events) / args.steps
    dec_ms = sum(e[1].elapsed_time(e[2]) for e in events) / args.steps

    # verification (outside the timed region): every status 0, exact sizes, exact bytes
    bad = int((est != 0).sum() + (bst != 0).sum() + (blens != lens).sum())
    bad += 0 if torch.equal(back, raw) else 1
    enc_bytes = int(elens.sum())
    elapsed = hcdist.reduce_counters([t1 - t0], op="max", device=dev)
    bad, enc_total = (int(v) for v in hcdist.reduce_counters([bad, enc_bytes], device=dev))
    sizes = hcdist.gather_sizes(elens)  # every stream's encoded size, on every rank
    gather_ms = None
    if args.gather:  # the encoded payloads of all ranks into rank 0 (RCCL all-gather)
        torch.cuda.synchronize(dev)
        g0 = time.perf_counter()
        packed, _ = hcdist.gather_encoded(enc, eoffs, elens)
        torch.cuda.synchronize(dev)
        gather_ms = (time.perf_counter() - g0) * 1e3
        if rank == 0 and packed.numel() != int(sizes.sum()):
            bad += 1
    if bad:
        raise SystemExit(f"bit-exact check FAILED on {bad} items")

    step_s = float(elapsed) / args.steps
    raw_total = world * S * N_RAW
    value = raw_total / step_s / 2**30
    # roofline of the dominant kernel: algorithmic bytes per launch (raw read + encoded written
    # for encode, encoded read + raw written for decode) / its average launch time
    alg_bytes = S * N_RAW + enc_bytes  # this rank, per launch
    dom, dom_ms = ("decode_kernel", dec_ms) if dec_ms >= enc_ms else ("encode_kernel", enc_ms)
    achieved = alg_bytes / (dom_ms * 1e-3) / 1e9
    traffic = None
    tpath = args.traffic or os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tpath):
        with open(tpath) as f:
            t = json.load(f)
        key = f"{dom}:{'cm' if use_diff else 'c'}:{args.kind}:{S}"
        traffic = t.get(key)
    # the issue bound of the dominant kernel, from its PMC instruction counts (profiles/, same
    # workload only) over this run's launch time
    issue = None
    ppath = os.path.join(ROOT, "profiles", "r01_pmc_summary.json")
    if use_diff and args.kind == "photo" and S == 8192 and os.path.exists(ppath):
        with open(ppath) as f:
            pm = json.load(f)
        ps = pm.get("per_symbol", {}).get({"encode_kernel": "encode_kernel<narrow,raw+diff>",
                                           "decode_kernel": "decode_kernel<narrow,raw>"}[dom])
        if ps:
            per_cu = (ps["SQ_INSTS_VALU"] + ps["SQ_INSTS_SALU"]) * pm["symbols_per_launch"] / 256
            ach = per_cu / (dom_ms * 1e-3 * CLOCK_HZ)
            issue = {"bound": "VALU+SALU issue", "kernel": dom, "achieved": round(ach, 3), "peak": ISSUE_PEAK,
                     "unit": "instructions/cycle/CU", "frac": round(ach / ISSUE_PEAK, 3),
                     "source": "profiles/r01_pmc_summary.json (SQ_INSTS_VALU+SQ_INSTS_SALU per symbol), "
                               "peak: scripts/micro/issue.hip"}
    result = {
        "metric": METRIC, "value": round(value, 4), "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": f"synthetic {args.kind} (SURVEY.md App. D, seed 0x5EED), generated in HBM",
        "config": {"workload": f"C5 shard: {S} x 512x512 {args.kind} streams per GPU, "
                               f"{'-c -m' if use_diff else '-c'} encode + decode round trip",
                   "streams_per_gpu": S, "stream_bytes": N_RAW, "mode": "-c -m" if use_diff else "-c",
                   "parallelism": f"dp{world} (stream shards, no data-path collective)"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 3), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 6), "traffic": traffic,
                     "alg_bytes_per_launch": alg_bytes, "avg_launch_ms": round(dom_ms, 4)},
        "issue": issue,
        "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4),
        "encode_GiBps": round(world * S * N_RAW / (enc_ms * 1e-3) / 2**30, 4),
        "decode_GiBps": round(world * S * N_RAW / (dec_ms * 1e-3) / 2**30, 4),
        "bits_per_byte": round(enc_total * 8 / raw_total, 4), "bit_exact": True,
        "streams_total": int(sizes.numel()),
    }
    if gather_ms is not None:
        result["gather_ms"] = round(gather_ms, 3)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cores = min(16, os.cpu_count() or 1)
        result["cpu_baseline"] = cpu_baseline(args, cores)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
