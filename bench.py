#!/usr/bin/env python3
"""bench.py — encode+decode GiB/s of the MI355X huffman-codec on batched 512x512 .raw streams.

Headline workload = BASELINE.json configs[4] (C5): ONE batch of 65536 synthetic 512x512 photo
streams (seed 0x5EED, generated in HBM), split over the N GPUs (strong
scaling, as BASELINE defines C5: rank r owns streams [r*S, (r+1)*S), S = 65536 / N; at N=8 each GPU
holds 8192 streams). The streams are independent units, so there is no data-path collective.
One step is the reference's full round trip on the shard: `-c -m` encode (diff -> MNP-5 RLE ->
FGK -> header, one fused kernel) then decode (FGK -> RLE revert -> diff revert, one fused kernel).
value = raw bytes of all ranks / step time (max over ranks), GiB/s. After the timed region: every
status 0, decode == input on every stream, and (rank 0, N=1) the first streams' encodings
byte-identical to the reference binary's own output for them.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

`--gpus N` with N > 1 and no launcher around the process starts the N ranks itself (fresh child
processes through torch.distributed.run, before anything here touches a GPU) and exits with their
status; under a launcher, --gpus must equal WORLD_SIZE. At N > 1 the line also carries
`weak_scaling`: every rank then codes a whole 65536-stream batch of its own (per-GPU work fixed),
measured after the headline and reported beside it, never as `value`. `--weak` makes --streams a
per-GPU count for the headline itself.

At N=1 the same JSON line also carries "configs": the other BASELINE.json configs measured in
the same run (C1 the per-file CLI, C2 one stream, C3 4096 streams `-c`, C4 the 4096x4096
adaptive matrix, the grad / noise distributions of SURVEY.md §8d, and C5_split2/4/8: the shard
one GPU holds when C5 is split over 2 / 4 / 8 GPUs, with its efficiency against the whole batch),
each checked against the reference's digests (tests/golden/digests.json) or by round trip. The
full per-config record (rooflines, adaptive stages, CLI phases) is printed first on a line of its
own starting with "detail "; the last line is the one JSON result.

Streams are independent, so ranks share nothing on the data path; after the timed region RCCL
all-reduces the verification counters and the max step time.
"""
import argparse
import hashlib
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
C5_STREAMS = 65536
PMC_PATH = os.path.join(ROOT, "profiles", "pmc_summary.json")
FGK_SRC = os.path.join(ROOT, "huffman-codec_amd", "csrc", "hc_fgk.hip")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--streams", "--total-streams", dest="streams", type=int, default=C5_STREAMS,
                    help="streams in the whole batch, split over the ranks (strong scaling; 65536 = C5)")
    ap.add_argument("--weak", action="store_true", help="--streams per GPU instead (weak scaling)")
    ap.add_argument("--no-weak-line", action="store_true",
                    help="N > 1: skip the extra weak-scaling measurement (a whole C5 batch per GPU)")
    ap.add_argument("--kind", default="photo", choices=["photo", "grad", "noise"])
    ap.add_argument("--no-diff", action="store_true", help="-c instead of -c -m")
    ap.add_argument("--cpu-sample", type=int, default=0, help="streams for the CPU baseline (0 = auto)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gather", action="store_true",
                    help="after the timed region: pack every rank's encoded shard on its GPU and send it to rank 0 "
                         "(the north star's final gather), timed and reported separately")
    ap.add_argument("--no-configs", action="store_true", help="N=1: skip the other BASELINE configs")
    ap.add_argument("--only-configs", default="", help="comma list: run just these configs (no headline)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL on ROCm): the GPU run; gloo: a CPU dry run of the multi-rank path "
                         "(sharding, barriers, timing, max-over-ranks, counter reduction, --gather) with a "
                         "stand-in per-rank step that copies each stream instead of coding it")
    ap.add_argument("--dry-stream-bytes", type=int, default=4096, help="gloo dry run: bytes per stream")
    return ap.parse_args(argv)


def sha(b):
    return hashlib.sha256(b).hexdigest()


def src_sha():
    with open(FGK_SRC, "rb") as f:
        return sha(f.read())[:16]


def host_cpus():
    """The host's CPUs: the model, the hardware threads and physical cores of the node, and how
    many this process may use (affinity and the cgroup CPU quota: a GPU box gives one GPU's job a
    share of the node's cores)"""
    info = {"cpu_model": "?", "node_threads": os.cpu_count() or 1}
    cores = set()
    try:
        phys = None
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "model name" and info["cpu_model"] == "?":
                    info["cpu_model"] = v
                elif k == "physical id":
                    phys = v
                elif k == "core id":
                    cores.add((phys, v))
    except OSError:
        pass
    info["physical_cores"] = len(cores) or info["node_threads"]
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = info["node_threads"]
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    info["affinity_threads"] = aff
    info["cgroup_cpu_quota"] = quota
    info["usable"] = max(1, min(aff, int(quota) if quota else aff))
    return info


def cpu_baseline(args, cores, gpu_encoded):
    """The reference binary itself (oracle/_ref: the Makefile build, -O0, and the same sources
    at -O2) on a bounded sample of the same workload, one process per stream over `cores` host
    cores. The sample is rank 0's first streams, so the reference's .huf files are also compared
    byte for byte with the GPU's encodings of the same streams (gpu_encoded)."""
    import subprocess
    from concurrent.futures import ThreadPoolExecutor

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    sample = min(args.cpu_sample or 8 * cores, len(gpu_encoded))
    raws = [oracle.synth(args.kind, k).tobytes() for k in range(sample)]
    mode = ["-c"] if args.no_diff else ["-c", "-m"]
    legs = []
    for label, binary in (("-O2", oracle.REF_BIN_O2), ("Makefile -O0", oracle.REF_BIN)):
        if not os.path.exists(binary):
            continue
        tmp = tempfile.mkdtemp(dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
        try:
            for i, r in enumerate(raws):
                with open(os.path.join(tmp, f"{i}.raw"), "wb") as f:
                    f.write(r)

            def enc(i):
                subprocess.run([binary] + mode + ["-i", f"{i}.raw", "-o", f"{i}.huf"], cwd=tmp, check=True,
                               capture_output=True)

            def dec(i):
                subprocess.run([binary, "-d", "-i", f"{i}.huf", "-o", f"{i}.out"], cwd=tmp, check=True,
                               capture_output=True)

            with ThreadPoolExecutor(cores) as ex:
                t0 = time.perf_counter()
                list(ex.map(enc, range(sample)))
                t1 = time.perf_counter()
                list(ex.map(dec, range(sample)))
                t2 = time.perf_counter()
            rt = all(open(os.path.join(tmp, f"{i}.out"), "rb").read() == raws[i] for i in range(sample))
            same = all(open(os.path.join(tmp, f"{i}.huf"), "rb").read() == gpu_encoded[i] for i in range(sample))
        finally:
            for fn in os.listdir(tmp):
                os.remove(os.path.join(tmp, fn))
            os.rmdir(tmp)
        total = sample * N_RAW
        legs.append({"build": label, "value": total / (t2 - t0) / 2**30, "encode_GiBps": total / (t1 - t0) / 2**30,
                     "decode_GiBps": total / (t2 - t1) / 2**30, "seconds": t2 - t0, "round_trip": rt,
                     "gpu_bytes_identical": same})
    if not legs:
        return None
    main_leg = legs[0]
    return {"value": main_leg["value"], "unit": "GiB/s", "cores": cores, "kind": "reference",
            "build": main_leg["build"],
            "sample": f"{sample} x 512x512 {args.kind} streams (k = 0..{sample - 1}), {' '.join(mode)} then -d, "
                      f"one process per stream on the {cores} host CPUs this job may use (oracle/_ref, compiled from the reference "
                      f"sources; value = the {main_leg['build']} build, every build in legs)",
            "legs": legs,
            "bit_exact_vs_gpu": all(l["gpu_bytes_identical"] and l["round_trip"] for l in legs)}


class Batch:
    """S synthetic 512x512 streams resident in HBM with encode / decode buffers."""

    def __init__(self, torch, hc, dev, kind, k0, S, use_diff, side=512, kinds=None):
        self.torch, self.hc, self.dev, self.S, self.use_diff = torch, hc, dev, S, use_diff
        self.N = side * side
        N = self.N
        self.cap = 2 * N + 4096
        self.raw = torch.empty(S * N, dtype=torch.uint8, device=dev)
        if kinds is None:
            hc.synth_batch(kind, k0, S, side, side, self.raw, N)
        else:  # [(kind, count), ...] one after another (a mixed batch)
            at = 0
            for kd, cnt in kinds:
                hc.synth_batch(kd, k0, cnt, side, side, self.raw[at * N:(at + cnt) * N], N)
                at += cnt
        i64 = dict(dtype=torch.int64, device=dev)
        self.offs = torch.arange(S, **i64) * N
        self.lens = torch.full((S,), N, **i64)
        self.enc = torch.empty(S * self.cap, dtype=torch.uint8, device=dev)
        self.eoffs = torch.arange(S, **i64) * self.cap
        self.ecaps = torch.full((S,), self.cap, **i64)
        self.elens = torch.zeros(S, **i64)
        self.est = torch.zeros(S, dtype=torch.int32, device=dev)
        self.back = torch.empty_like(self.raw)
        self.blens = torch.zeros_like(self.lens)
        self.bst = torch.zeros_like(self.est)

    def step(self, stream, ev=None):
        hc = self.hc
        if ev is not None:
            ev[0].record(stream)
        hc.compress_batch(self.raw, self.offs, self.lens, self.enc, self.eoffs, self.ecaps, self.elens,
                          self.est, use_diff=self.use_diff, stream=stream)
        if ev is not None:
            ev[1].record(stream)
        hc.decompress_batch(self.enc, self.eoffs, self.elens, self.back, self.offs, self.lens, self.blens,
                            self.bst, stream=stream)
        if ev is not None:
            ev[2].record(stream)

    def bad(self):
        torch = self.torch
        b = int((self.est != 0).sum() + (self.bst != 0).sum() + (self.blens != self.lens).sum())
        return b + (0 if torch.equal(self.back, self.raw) else 1)

    def fgk_symbols(self):
        """FGK symbols of the whole batch: every stream's u64 header count (headers.cpp:110-116)"""
        t = self.torch
        hdr = self.enc[self.eoffs.view(-1, 1) + t.arange(8, device=self.enc.device)].to(t.int64)
        return int((hdr << (8 * t.arange(8, device=self.enc.device))).sum())

    def encoded(self, k):
        n = int(self.elens[k])
        o = k * self.cap
        return self.enc[o:o + n].cpu().numpy().tobytes()


class HostEvent:
    """torch.cuda.Event's record / elapsed_time on the host clock (the gloo dry run)"""

    def __init__(self, **_):
        self.t = None

    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


def sync(torch, dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def timed(torch, b, stream, steps, warmup, barrier=None):
    """warmup + `steps` timed round trips; returns (wall seconds, enc ms, dec ms per launch)"""
    for _ in range(warmup):
        b.step(stream)
    sync(torch, b.dev)
    Ev = torch.cuda.Event if b.dev.type == "cuda" else HostEvent
    events = [[Ev(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    if barrier:
        barrier()
    sync(torch, b.dev)
    t0 = time.perf_counter()
    for k in range(steps):
        b.step(stream, events[k])
    sync(torch, b.dev)
    if barrier:
        barrier()
    t1 = time.perf_counter()
    enc_ms = sum(e[0].elapsed_time(e[1]) for e in events) / steps
    dec_ms = sum(e[1].elapsed_time(e[2]) for e in events) / steps
    return t1 - t0, enc_ms, dec_ms


def roofline(S, N, enc_bytes, enc_ms, dec_ms, mode, kind):
    """the dominant kernel: algorithmic bytes per launch (raw read + encoded written for encode,
    encoded read + raw written for decode) / its average launch time (HIP events
    on the launch stream); traffic = PMC HBM bytes per launch from profiles/pmc_summary.json when
    that file was measured on this exact kernel source and workload"""
    alg = S * N + enc_bytes
    dom, ms = ("decode_kernel", dec_ms) if dec_ms >= enc_ms else ("encode_kernel", enc_ms)
    ach = alg / (ms * 1e-3) / 1e9
    r = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 3), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
         "frac": round(ach / HBM_PEAK_GBPS, 6), "traffic": None, "alg_bytes_per_launch": alg,
         "avg_launch_ms": round(ms, 4)}
    issue = None
    if os.path.exists(PMC_PATH):
        with open(PMC_PATH) as f:
            pm = json.load(f)
        # each stream is coded by one launch of the kernel's family (path cache / level tables /
        # small alphabet): the workload's counters are their sum
        keys = [f"{dom}{v}:{mode}:{kind}:{S}" for v in ("", "_tables", "_small")]
        parts = [pm.get("launches", {}).get(k) for k in keys]
        key = " + ".join(k for k, p in zip(keys, parts) if p)
        e = None
        if key:
            e = {c: sum(p.get(c, 0) for p in parts if p) for c in ("hbm_bytes", "valu_salu_insts")
                 if all(c in p for p in parts if p)}
        if e and pm.get("source_sha") == src_sha():
            r["traffic"] = e.get("hbm_bytes")
            r["traffic_source"] = f"profiles/pmc_summary.json[{key}] (rocprofv3 PMC, same kernel source)"
            if "valu_salu_insts" in e:
                ach_i = e["valu_salu_insts"] / 256 / (ms * 1e-3 * CLOCK_HZ)
                issue = {"bound": "VALU+SALU issue", "kernel": dom, "achieved": round(ach_i, 3), "peak": ISSUE_PEAK,
                         "unit": "instructions/cycle/CU", "frac": round(ach_i / ISSUE_PEAK, 3),
                         "source": f"SQ_INSTS_VALU+SQ_INSTS_SALU per launch from profiles/pmc_summary.json[{key}]; "
                                   "peak: scripts/micro/issue.hip"}
    return r, issue


def config_batch(torch, hc, dev, stream, name, what, kind, S, use_diff, steps, digests, side=512):
    b = Batch(torch, hc, dev, kind, 0, S, use_diff, side)
    wall, enc_ms, dec_ms = timed(torch, b, stream, steps, 1)
    bad = b.bad()
    mode = "cm" if use_diff else "c"
    enc_bytes = int(b.elens.sum())
    out = {"what": what, "streams": S, "mode": "-c -m" if use_diff else "-c", "kind": kind,
           "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4),
           "GiBps": round(S * b.N / ((enc_ms + dec_ms) * 1e-3) / 2**30, 4),
           "encode_GiBps": round(S * b.N / (enc_ms * 1e-3) / 2**30, 4),
           "decode_GiBps": round(S * b.N / (dec_ms * 1e-3) / 2**30, 4),
           "bits_per_byte": round(enc_bytes * 8 / (S * b.N), 4), "round_trip_exact": bad == 0,
           "fgk_symbols_per_stream": round(b.fgk_symbols() / S, 1)}
    # the reference's digests for streams k = 0..3 of this kind (512x512)
    if side == 512 and digests:
        ok = True
        for k in range(min(S, 4)):
            want = digests["synthetic"][f"{kind}_{k}"][mode]
            got = b.encoded(k)
            ok &= (len(got), sha(got)) == (want["len"], want["sha256"])
        out["reference_digests_identical"] = bool(ok)
        bad += 0 if ok else 1
    out["roofline"], out["issue"] = roofline(S, b.N, enc_bytes, enc_ms, dec_ms, mode, kind)
    del b
    torch.cuda.empty_cache()
    return out, bad


class AdaptBatch:
    """S synthetic side x side matrices resident in HBM, coded with -c -a [-m] through the batched
    adaptive API (hc_compress_adapt_batch / hc_decompress_adapt_batch), workspaces preallocated"""

    def __init__(self, torch, hc, dev, kind, S, use_diff, side):
        self.torch, self.hc, self.dev, self.S, self.use_diff = torch, hc, dev, S, use_diff
        self.N = side * side
        N = self.N
        self.cap = 2 * N + 4096 if side <= 512 else (hc.compress_bound(N, True) + 255) // 256 * 256
        self.raw = torch.empty(S * N, dtype=torch.uint8, device=dev)
        hc.synth_batch(kind, 0, S, side, side, self.raw, N)
        i64 = dict(dtype=torch.int64, device=dev)
        self.offs = torch.arange(S, **i64) * N
        self.lens = torch.full((S,), N, **i64)
        self.widths = torch.full((S,), side, **i64)
        self.enc = torch.empty(S * self.cap, dtype=torch.uint8, device=dev)
        self.eoffs = torch.arange(S, **i64) * self.cap
        self.ecaps = torch.full((S,), self.cap, **i64)
        self.elens = torch.zeros(S, **i64)
        self.est = torch.zeros(S, dtype=torch.int32, device=dev)
        self.back = torch.empty_like(self.raw)
        self.blens = torch.zeros_like(self.lens)
        self.bst = torch.zeros_like(self.est)
        L = hc.lib()
        self.wenc = torch.empty(int(L.hc_adapt_compress_work_bound(S * N, S)), dtype=torch.uint8, device=dev)
        # the decode workspace is sized from the encoded lengths: one untimed encode first
        hc.compress_adapt_batch(self.raw, self.offs, self.lens, self.widths, self.enc, self.eoffs, self.ecaps,
                                self.elens, self.est, use_diff=use_diff, work=self.wenc)
        torch.cuda.synchronize(dev)
        self.wdec = torch.empty(int(L.hc_adapt_decompress_work_bound(int(self.elens.sum()), S * N, S)),
                                dtype=torch.uint8, device=dev)

    def step(self, stream, ev=None):
        hc = self.hc
        if ev is not None:
            ev[0].record(stream)
        hc.compress_adapt_batch(self.raw, self.offs, self.lens, self.widths, self.enc, self.eoffs, self.ecaps,
                                self.elens, self.est, use_diff=self.use_diff, stream=stream, work=self.wenc)
        if ev is not None:
            ev[1].record(stream)
        hc.decompress_adapt_batch(self.enc, self.eoffs, self.elens, self.back, self.offs, self.lens, self.blens,
                                  self.bst, stream=stream, work=self.wdec)
        if ev is not None:
            ev[2].record(stream)

    bad = Batch.bad
    encoded = Batch.encoded


# algorithmic bytes of the adaptive stages that stream data (raw: matrix bytes, syms: adaptive
# symbol bytes): what each must read and write at least
ADAPT_STAGE_BYTES = {"tile_cost": lambda raw, syms: raw, "emit_tile": lambda raw, syms: raw + syms,
                     "bounds": lambda raw, syms: syms, "unblock_tile": lambda raw, syms: syms + raw,
                     "chunk_sum": lambda raw, syms: raw, "undiff": lambda raw, syms: 2 * raw}


def adapt_stages(torch, hc, b, stream):
    """one more encode + decode with the library's stage clock on (HIP events on the launch stream
    after every stage): each stage's time, and for the streaming stages their algorithmic bytes
    over that time against the HBM peak (8 TB/s)"""
    hc.use_debug_build(True)  # the stage clock exists in the debug build only
    hc.debug_stage_clock(True)
    try:
        hc.compress_adapt_batch(b.raw, b.offs, b.lens, b.widths, b.enc, b.eoffs, b.ecaps, b.elens, b.est,
                                use_diff=b.use_diff, stream=stream, work=b.wenc)
        enc = hc.debug_stage_times()
        hc.decompress_adapt_batch(b.enc, b.eoffs, b.elens, b.back, b.offs, b.lens, b.blens, b.bst,
                                  stream=stream, work=b.wdec)
        dec = hc.debug_stage_times()
    finally:
        hc.debug_stage_clock(False)
        hc.use_debug_build(False)
    torch.cuda.synchronize(b.dev)
    raw = b.S * b.N
    # adaptive symbols per stream: the FGK header's u64 count, the first 8 bytes of each stream
    hdr = b.enc[b.eoffs.view(-1, 1) + torch.arange(8, device=b.dev)].to(torch.int64)
    syms = int((hdr << (8 * torch.arange(8, device=b.dev))).sum())
    out = {"adaptive_symbol_bytes": syms}
    for direction, stages in (("encode", enc), ("decode", dec)):
        d = {}
        for name, ms in stages:
            e = {"ms": round(ms, 4)}
            if name in ADAPT_STAGE_BYTES and ms > 0:
                nb = ADAPT_STAGE_BYTES[name](raw, syms)
                gbs = nb / (ms * 1e-3) / 1e9
                e.update({"alg_bytes": nb, "GBps": round(gbs, 1), "hbm_frac": round(gbs / 8000.0, 4)})
            d[name] = e
        if direction == "decode":  # the serial and the parallel boundary passes together
            ms = sum(v["ms"] for k, v in d.items() if k == "bounds" or k.startswith("par_"))
            if ms > 0:
                gbs = syms / (ms * 1e-3) / 1e9
                d["block_boundaries"] = {"ms": round(ms, 4), "alg_bytes": syms, "GBps": round(gbs, 1),
                                         "hbm_frac": round(gbs / 8000.0, 4),
                                         "stages": "bounds + par_fsm/entry/z/scan/walk/fix"}
        out[direction] = d
    return out


def config_adapt(torch, hc, dev, stream, what, S, side, use_diff, steps, digests):
    """-c -a [-m] on S side x side photo matrices, device-resident, batched adaptive API; checked
    against the reference's digests (512x512 k = 0..3, or the 4096x4096 matrix) and by round trip"""
    b = AdaptBatch(torch, hc, dev, "photo", S, use_diff, side)
    wall, enc_ms, dec_ms = timed(torch, b, stream, steps, 1)
    bad = b.bad()
    mode = "cma" if use_diff else "ca"
    ok = True
    for k in range(min(S, 4)):
        want = digests["synthetic"][f"photo_{k}"][mode] if side == 512 else digests["synthetic_4096"]["photo_0"][mode]
        got = b.encoded(k)
        ok &= (len(got), sha(got)) == (want["len"], want["sha256"])
    bad += 0 if ok else 1
    enc_bytes = int(b.elens.sum())
    out = {"what": what, "streams": S, "mode": "-c -a -m" if use_diff else "-c -a", "kind": "photo",
           "side": side, "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4),
           "GiBps": round(S * b.N / ((enc_ms + dec_ms) * 1e-3) / 2**30, 4),
           "encode_GiBps": round(S * b.N / (enc_ms * 1e-3) / 2**30, 4),
           "decode_GiBps": round(S * b.N / (dec_ms * 1e-3) / 2**30, 4),
           "bits_per_byte": round(enc_bytes * 8 / (S * b.N), 4), "round_trip_exact": b.bad() == 0,
           "reference_digests_identical": bool(ok), "stages": adapt_stages(torch, hc, b, stream)}
    del b
    torch.cuda.empty_cache()
    return out, bad


def config_mixed(torch, hc, dev, stream, photos=6144, noises=2048):
    """a batch mixing two alphabets (photo -c -m: the encoder's path cache; noise -c -m: its level
    tables), encoded as one batch and as its two parts: each stream's mode is its own and the
    two modes' launches run side by side, so the mixed batch should cost no more than the parts"""
    out, bad = {"what": f"{photos} photo + {noises} noise 512x512 -c -m in one batch vs the two parts", "mode": "-c -m"}, 0
    for name, kinds, S in (("mixed", [("photo", photos), ("noise", noises)], photos + noises),
                           ("photo_part", None, photos), ("noise_part", None, noises)):
        kind = "noise" if name == "noise_part" else "photo"
        b = Batch(torch, hc, dev, kind, 0, S, True, kinds=kinds)
        _, enc_ms, dec_ms = timed(torch, b, stream, 2, 1)
        bad += b.bad()
        out[name] = {"streams": S, "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4)}
        del b
        torch.cuda.empty_cache()
    out["encode_mixed_over_parts"] = round(out["mixed"]["encode_ms"] /
                                           (out["photo_part"]["encode_ms"] + out["noise_part"]["encode_ms"]), 4)
    out["round_trip_exact"] = bad == 0
    return out, bad


CLI_BIN = os.path.join(ROOT, "huffman-codec_amd", "bin", "huffman-codec")
FLOOR_BIN = os.path.join(ROOT, "huffman-codec_amd", "bin", "hc-floor")


def _hc_times(stderr):
    for line in stderr.decode(errors="replace").splitlines():
        if line.startswith("hc-times "):
            return {k: float(v) for k, v in (f.split("=") for f in line.split()[1:])}
    return None


def config_cli(reps=7):
    """C1 (BASELINE configs[0]): the drop-in CLI per file, the reference's own use case (one file
    per process, main.cpp:152-221): hd01.raw `-c -m` then `-d`, wall clock per process including
    its start, for this repo's GPU CLI and for the reference binary (oracle/_ref, -O2 and the
    Makefile's -O0), median of `reps` runs each. hd01.raw is recovered on the box by decoding the
    reference's committed output tests/golden/corpus/hd01.cm.huf with the reference binary; every
    binary's .huf must equal that file and every decode must give hd01.raw back.

    The floor: bin/hc-floor, an empty HIP program (process start, HIP start-up, one empty kernel
    launched and waited for) timed the same way on the same box; `cli_minus_floor_ms` is what the
    CLI costs per file above what any GPU process costs. The GPU CLI also reports its in-process
    phases (HC_CLI_TIMES=1: read, HIP start-up, coding, write), so its wall time splits into process
    start + library load, HIP start-up and coding, and the coding into its one-time part (code
    objects loaded at the first launch, first allocations) and the rest (code_again_ms: the same
    call repeated in the process, i.e. copies in and out plus kernels). The phase runs are separate
    from the wall-clock runs (they code twice). A failing binary is recorded in the entry (and
    counted bad) instead of aborting the other configs."""
    import statistics
    import subprocess

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    ref = oracle.REF_BIN_O2 if os.path.exists(oracle.REF_BIN_O2) else oracle.REF_BIN
    golden = os.path.join(ROOT, "tests", "golden", "corpus", "hd01.cm.huf")
    if not (os.path.exists(ref) and os.path.exists(CLI_BIN)):
        return {"what": "C1 hd01 -c -m per file", "skipped": "reference binary or GPU CLI not built"}, 0
    want = open(golden, "rb").read()
    tmp = tempfile.mkdtemp(dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    bad = 0
    out = {"what": "C1: hd01.raw -c -m then -d, one process per file (the reference's use case), "
                   f"median of {reps} runs, wall clock including process start", "binaries": {}}
    try:
        r = subprocess.run([ref, "-d", "-i", golden, "-o", "hd01.raw"], cwd=tmp, capture_output=True)
        if r.returncode != 0:
            out["error"] = f"reference decode of hd01.cm.huf: exit {r.returncode}"
            return out, 1
        raw = open(os.path.join(tmp, "hd01.raw"), "rb").read()
        out["file_bytes"] = len(raw)
        if os.path.exists(FLOOR_BIN):
            walls, phases, err = [], [], None
            for rep in range(2 * reps):
                timing = rep >= reps
                env = dict(os.environ, HC_CLI_TIMES="1") if timing else None
                t0 = time.perf_counter()
                r = subprocess.run([FLOOR_BIN], cwd=tmp, capture_output=True, env=env)
                if r.returncode != 0:
                    err = f"exit {r.returncode}: {r.stderr[-200:]!r}"
                    break
                if timing:
                    p = _hc_times(r.stderr)
                    if p:
                        phases.append(p)
                else:
                    walls.append(time.perf_counter() - t0)
            if err:
                out["floor"] = {"error": err}
            else:
                fl = {"binary": os.path.relpath(FLOOR_BIN, ROOT), "wall_s": round(statistics.median(walls), 4)}
                if phases:
                    fl["phases_ms"] = {k: round(statistics.median(p[k] for p in phases), 3) for k in phases[0]}
                out["floor"] = fl
        legs = [("gpu_cli", CLI_BIN), ("reference_O2", oracle.REF_BIN_O2), ("reference_O0", oracle.REF_BIN)]
        for label, binary in legs:
            if not os.path.exists(binary):
                continue
            enc_t, dec_t, phases = [], [], {"encode": [], "decode": []}
            same = rt = True
            err = None
            for rep in range(2 * reps if label == "gpu_cli" else reps):
                timing = rep >= reps  # the GPU CLI's phase runs come after its wall-clock runs
                env = dict(os.environ, HC_CLI_TIMES="1") if timing else None
                for d, cmd, t in (("encode", ["-c", "-m", "-i", "hd01.raw", "-o", f"{label}.huf"], enc_t),
                                  ("decode", ["-d", "-i", f"{label}.huf", "-o", f"{label}.out"], dec_t)):
                    t0 = time.perf_counter()
                    r = subprocess.run([binary] + cmd, cwd=tmp, capture_output=True, env=env)
                    if not timing:
                        t.append(time.perf_counter() - t0)
                    if r.returncode != 0:
                        err = f"{d}: exit {r.returncode}: {r.stderr[-300:]!r}"
                        break
                    p = _hc_times(r.stderr)
                    if p:
                        phases[d].append(p)
                if err:
                    break
                same &= open(os.path.join(tmp, f"{label}.huf"), "rb").read() == want
                rt &= open(os.path.join(tmp, f"{label}.out"), "rb").read() == raw
            if err:
                out["binaries"][label] = {"binary": os.path.relpath(binary, ROOT), "error": err}
                bad += 1
                continue
            leg = {"binary": os.path.relpath(binary, ROOT), "encode_s": round(statistics.median(enc_t), 4),
                   "decode_s": round(statistics.median(dec_t), 4), "encode_bytes_identical_to_reference": bool(same),
                   "round_trip": bool(rt)}
            for d in ("encode", "decode"):
                if phases[d]:
                    med = {k: round(statistics.median(p[k] for p in phases[d]), 3) for k in phases[d][0]}
                    wall_ms = leg[f"{d}_s"] * 1e3
                    med["process_start_and_load_ms"] = round(
                        wall_ms - sum(v for k, v in med.items() if k != "code_again_ms"), 3)
                    leg[f"{d}_phases_ms"] = med
            out["binaries"][label] = leg
            bad += 0 if (same and rt) else 1
        g, r2 = out["binaries"].get("gpu_cli"), out["binaries"].get("reference_O2")
        if g and r2 and "encode_s" in g and "encode_s" in r2:
            out["gpu_over_reference_O2"] = {"encode": round(g["encode_s"] / r2["encode_s"], 3),
                                            "decode": round(g["decode_s"] / r2["decode_s"], 3)}
        fl = out.get("floor", {})
        if g and "encode_s" in g and "wall_s" in fl:
            out["cli_minus_floor_ms"] = {"encode": round((g["encode_s"] - fl["wall_s"]) * 1e3, 1),
                                         "decode": round((g["decode_s"] - fl["wall_s"]) * 1e3, 1)}
    except (OSError, subprocess.SubprocessError) as e:
        out["error"] = repr(e)[:300]
        bad += 1
    finally:
        for fn in os.listdir(tmp):
            os.remove(os.path.join(tmp, fn))
        os.rmdir(tmp)
    return out, bad


def run_configs(torch, hc, dev, stream, only, c5_kernel_GiBps=None):
    with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
        digests = json.load(f)
    plan = [
        ("C2", "1 x 512x512 photo -c -m: one stream, one wavefront (latency)", "photo", 1, True, 3),
        ("C3", "4096 x 512x512 photo -c", "photo", 4096, False, 3),
        ("grad", "8192 x 512x512 grad -c -m (best case: runs collapse the symbols)", "grad", 8192, True, 3),
        ("noise", "2048 x 512x512 noise -c -m (worst case: ~262k deep codes per stream)", "noise", 2048, True, 2),
    ]
    # C5 split over 2 / 4 / 8 GPUs: the shard each GPU holds, coded here on one GPU. Its kernel
    # throughput over the whole batch's is the strong-scaling efficiency ceiling at that N (the
    # shards are independent; what one GPU does with 65536 / N streams is what each of N does)
    for n in (2, 4, 8):
        plan.append((f"C5_split{n}", f"{C5_STREAMS // n} x 512x512 photo -c -m: the shard of one GPU when C5 is "
                                     f"split over {n} GPUs", "photo", C5_STREAMS // n, True, 3))
    res, bad = {}, 0
    if not only or "C1" in only:
        res["C1"], bad = config_cli()
    for name, what, kind, S, d, steps in plan:
        if only and name not in only:
            continue
        res[name], b = config_batch(torch, hc, dev, stream, name, what, kind, S, d, steps, digests)
        if name.startswith("C5_split") and c5_kernel_GiBps:
            res[name]["kernel_GiBps_C5"] = round(c5_kernel_GiBps, 4)
            res[name]["efficiency_vs_C5"] = round(res[name]["GiBps"] / c5_kernel_GiBps, 4)
        bad += b
    if not only or "mixed" in only:
        res["mixed"], b = config_mixed(torch, hc, dev, stream)
        bad += b
    aplan = [
        ("C4", "1 x 4096x4096 photo -c -a -w 4096 (one matrix: one FGK wavefront), device-resident", 1, 4096, False, 2),
        ("C4m", "1 x 4096x4096 photo -c -a -m -w 4096, device-resident", 1, 4096, True, 2),
        ("A512", "8192 x 512x512 photo -c -a -m (the reference's best-bpc mode), batched adaptive API", 8192, 512,
         True, 3),
    ]
    for name, what, S, side, d, steps in aplan:
        if only and name not in only:
            continue
        res[name], b = config_adapt(torch, hc, dev, stream, what, S, side, d, steps, digests)
        bad += b
    return res, bad


def copy_peak(torch, dev, stream, nbytes=1 << 30, reps=5):
    """measured HBM reference point next to the 8 TB/s datasheet peak: a 1 GiB
    device-to-device tensor copy, (read + write bytes) / best time, GB/s"""
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    best = None
    with torch.cuda.stream(stream):
        for _ in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            dst.copy_(src)
            e1.record(stream)
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
    del src, dst
    return round(2 * nbytes / (best * 1e-3) / 1e9, 1)


class StandInBatch:
    """The gloo dry run's per-rank work: S host streams of N pseudo-random bytes (stream k seeded by
    its global index k) with the same buffers, offsets and bookkeeping as Batch, whose step COPIES
    each stream into its encode slot and back instead of coding it. It exercises bench.py's
    multi-rank path (shards, barriers, timing, reductions, --gather) without a GPU; its numbers
    measure nothing about the codec."""

    def __init__(self, torch, k0, S, N):
        self.torch, self.dev, self.S, self.N = torch, torch.device("cpu"), S, N
        self.cap = N + 64
        self.raw = torch.cat([stand_in_stream(torch, k, N) for k in range(k0, k0 + S)]) if S else \
            torch.empty(0, dtype=torch.uint8)
        i64 = dict(dtype=torch.int64)
        self.offs = torch.arange(S, **i64) * N
        self.lens = torch.full((S,), N, **i64)
        self.enc = torch.zeros(S * self.cap, dtype=torch.uint8)
        self.eoffs = torch.arange(S, **i64) * self.cap
        self.elens = torch.zeros(S, **i64)
        self.back = torch.empty_like(self.raw)
        self.blens = torch.zeros_like(self.lens)

    def step(self, stream, ev=None):
        encv = self.enc.view(self.S, self.cap)
        if ev is not None:
            ev[0].record(stream)
        encv[:, :self.N] = self.raw.view(self.S, self.N)
        self.elens.fill_(self.N)
        if ev is not None:
            ev[1].record(stream)
        self.back.view(self.S, self.N)[:] = encv[:, :self.N]
        self.blens.copy_(self.elens)
        if ev is not None:
            ev[2].record(stream)

    def bad(self):
        return int((self.blens != self.lens).sum()) + (0 if self.torch.equal(self.back, self.raw) else 1)

    def fgk_symbols(self):
        return 0


def stand_in_stream(torch, k, N):
    """stream k of the gloo dry run: N bytes from a generator seeded with k"""
    g = torch.Generator().manual_seed(0x5EED + k)
    return torch.randint(0, 256, (N,), generator=g, dtype=torch.int64).to(torch.uint8)


def time_gather(torch, hcdist, b, dev, barrier):
    """every rank's encoded streams packed back to back on its GPU (hc_pack_batch), then sent to
    rank 0 point to point; max over ranks of the wall time; rank 0 checks the bytes it got"""
    ms = []
    for _ in range(2):
        if barrier:
            barrier()
        sync(torch, dev)
        t0 = time.perf_counter()
        packed, sizes = hcdist.gather_encoded(b.enc, b.eoffs, b.elens)
        sync(torch, dev)
        if barrier:
            barrier()
        ms.append((time.perf_counter() - t0) * 1e3)
    ms = float(hcdist.reduce_counters([min(ms)], op="max", device=dev)[0])
    total = int(sizes.sum())
    out = {"bytes_to_rank0": total, "ms": round(ms, 3), "GBps": round(total / (ms * 1e-3) / 1e9, 2),
           "how": "hc_pack_batch on each GPU, then batch_isend_irecv to rank 0 (RCCL p2p over xGMI)"
           if dev.type == "cuda" else "host packing, then batch_isend_irecv to rank 0 (gloo dry run)"}
    if packed is not None:
        out["packed_sha256"] = sha(packed.cpu().numpy().tobytes())
    if packed is not None:
        k = b.S - 1  # rank 0's own last stream sits at the end of its shard in the packed buffer
        at = int(b.elens[:k].sum())
        out["rank0_spot_check"] = bool(torch.equal(packed[at:at + int(b.elens[k])],
                                                   b.enc[int(b.eoffs[k]):int(b.eoffs[k]) + int(b.elens[k])]))
    return out


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args, argv):
    """--gpus N > 1 and no launcher around this process: start the N ranks (one per GPU) as fresh
    child processes through torch.distributed.run, rendezvous on 127.0.0.1, before anything in this
    process touches a GPU (no hcodec import, no HIP call: the children start from scratch); their
    output passes straight through and their exit status is returned. Under a launcher (WORLD_SIZE
    set) --gpus must equal the launcher's world size: a mismatch exits non-zero instead of measuring
    some other number of GPUs. Returns None when this process is itself the (only) rank."""
    import subprocess
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)", file=sys.stderr, flush=True)
            raise SystemExit(2)
        return None
    if args.gpus <= 1:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(cmd, env=env).returncode


def workload_name(total, world, S, kind, use_diff, weak):
    mode = "-c -m" if use_diff else "-c"
    how = (f"{S} per GPU, weak scaling" if weak else f"split over {world} GPU(s), {S} per GPU")
    c5 = total == C5_STREAMS and not weak and kind == "photo" and use_diff
    return (f"{'C5: ' if c5 else ''}{total} x 512x512 {kind} streams ({how}), {mode} encode + decode round trip")


def weak_line(torch, hc, hcdist, args, dev, stream, rank, world, barrier, dry, use_diff, N):
    """N > 1: every rank codes a whole batch of its own (C5's 65536 streams; the dry run: --streams),
    streams k = r*S .. r*S + S - 1, timed like the headline (max over ranks), verified the same way.
    Per-GPU work fixed: the weak-scaling figure, reported beside `value`, never as it."""
    S = args.streams if dry else C5_STREAMS
    steps = max(1, min(args.steps, 3))
    b = StandInBatch(torch, rank * S, S, N) if dry else Batch(torch, hc, dev, args.kind, rank * S, S, use_diff)
    wall, enc_ms, dec_ms = timed(torch, b, stream, steps, 1, barrier)
    bad = b.bad()
    del b
    if not dry:
        torch.cuda.empty_cache()
    elapsed = float(hcdist.reduce_counters([wall], op="max", device=dev)[0])
    bad = int(hcdist.reduce_counters([bad], device=dev)[0])
    if bad:
        raise SystemExit(f"weak-scaling pass: bit-exact check FAILED on {bad} items")
    step_s = elapsed / steps
    return {"what": "every rank codes a whole batch of its own (per-GPU work fixed); beside value, not value",
            "scaling": "weak", "streams_per_gpu": S, "streams_total": world * S, "steps": steps,
            "ms_per_step": round(step_s * 1e3, 3), "value": round(world * S * N / step_s / 2**30, 4),
            "unit": "GiB/s", "bit_exact": True}


# keys of a config's record kept in the final JSON line (the full record goes on the "detail" line)
_KEEP = ("streams", "mode", "kind", "encode_ms", "decode_ms", "GiBps", "round_trip_exact",
         "reference_digests_identical", "fgk_symbols_per_stream", "efficiency_vs_C5",
         "kernel_GiBps_C5", "encode_mixed_over_parts", "skipped")


def compact_configs(configs):
    out = {}
    for name, c in configs.items():
        d = {k: c[k] for k in _KEEP if k in c}
        if isinstance(c.get("roofline"), dict):
            d["hbm_frac"] = c["roofline"].get("frac")
        if isinstance(c.get("issue"), dict):
            d["issue_frac"] = c["issue"].get("frac")
        st = c.get("stages")
        if isinstance(st, dict):
            d["stages_ms"] = {k: v["ms"] for part in ("encode", "decode") for k, v in st.get(part, {}).items()
                              if k in ("tile_cost", "emit_tile", "unblock_tile", "block_boundaries", "undiff",
                                       "fgk_encode", "fgk_decode")}
        if name == "C1":
            for k in ("floor", "cli_minus_floor_ms", "gpu_over_reference_O2", "error"):
                if k in c:
                    d[k] = c[k]
            d["binaries"] = {b: {k: v[k] for k in ("encode_s", "decode_s", "encode_bytes_identical_to_reference",
                                                    "round_trip") if k in v}
                             for b, v in c.get("binaries", {}).items()}
        out[name] = d
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    rc = launch_ranks(args, argv)
    if rc is not None:
        raise SystemExit(rc)
    import torch
    import torch.distributed as dist
    import hcdist
    import hcodec as hc

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dry = args.backend == "gloo"  # the CPU dry run of this same path (StandInBatch per rank)
    # under torch.distributed.run (LOCAL_WORLD_SIZE set) the process group exists at every world
    # size, world 1 included: a one-GPU box then runs the RCCL init and collectives of the N-GPU path
    launched = world > 1 or "LOCAL_WORLD_SIZE" in os.environ
    if dry:
        if launched:
            dist.init_process_group("gloo")
        dev, stream = torch.device("cpu"), None
    else:
        if launched:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dev = torch.device("cuda", local)
        if not hc.device_ok():
            raise SystemExit("libhcodec.so: no usable gfx950 device")
        stream = torch.cuda.current_stream(dev)

    if args.only_configs and not dry:
        res, bad = run_configs(torch, hc, dev, stream, set(args.only_configs.split(",")))
        print(json.dumps({"configs": res, "bad": bad}), flush=True)
        raise SystemExit(1 if bad else 0)

    if args.weak:
        S = args.streams
    else:
        if args.streams % world:
            raise SystemExit(f"--streams {args.streams} does not split over {world} ranks")
        S = args.streams // world
    total = world * S
    use_diff = not args.no_diff
    N = args.dry_stream_bytes if dry else N_RAW
    b = StandInBatch(torch, rank * S, S, N) if dry else Batch(torch, hc, dev, args.kind, rank * S, S, use_diff)
    barrier = dist.barrier if dist.is_initialized() else None
    wall, enc_ms, dec_ms = timed(torch, b, stream, args.steps, args.warmup, barrier)

    # verification (outside the timed region): every status 0, exact sizes, exact bytes
    bad = b.bad()
    enc_bytes = int(b.elens.sum())
    elapsed = hcdist.reduce_counters([wall], op="max", device=dev)
    bad, enc_total = (int(v) for v in hcdist.reduce_counters([bad, enc_bytes], device=dev))
    if bad:
        raise SystemExit(f"bit-exact check FAILED on {bad} items")

    step_s = float(elapsed) / args.steps
    raw_total = world * S * N
    value = raw_total / step_s / 2**30
    mode = "cm" if use_diff else "c"
    roof, issue = (None, None) if dry else roofline(S, N, enc_bytes, enc_ms, dec_ms, mode, args.kind)
    result = {
        "metric": METRIC, "value": round(value, 4), "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 3),
        "higher_is_better": True, "scaling": "weak" if args.weak else "strong", "vs_baseline": None, "dtype": "u8",
        "data": f"synthetic {args.kind} (SURVEY.md App. D, seed 0x5EED), generated in HBM",
        "config": {"workload": workload_name(total, world, S, args.kind, use_diff, args.weak),
                   "streams_total": total, "streams_per_gpu": S, "stream_bytes": N,
                   "mode": "-c -m" if use_diff else "-c",
                   "parallelism": f"dp{world} (stream shards, no data-path collective)"},
        "roofline": roof, "issue": issue,
        "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4),
        "encode_GiBps": round(world * S * N / (enc_ms * 1e-3) / 2**30, 4) if enc_ms > 0 else None,
        "decode_GiBps": round(world * S * N / (dec_ms * 1e-3) / 2**30, 4) if dec_ms > 0 else None,
        "bits_per_byte": round(enc_total * 8 / raw_total, 4), "bit_exact": True,
        "fgk_symbols_per_stream": round(b.fgk_symbols() / S, 1) if S else None,
    }
    if dry:
        result.update({"metric": METRIC + " [gloo dry run: streams copied, not coded]", "dry_run": True,
                       "backend": "gloo", "bit_exact": None, "fgk_symbols_per_stream": None,
                       "data": "stand-in: pseudo-random bytes per stream (torch generator seeded by the stream index)"})
        result["config"]["workload"] = f"dry run: {total} x {N}-byte streams over {world} rank(s) ({S} per rank)"
    if dist.is_initialized():
        result["process_group"] = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    if world == 1 and not dry:
        roof["measured_copy_GBps"] = copy_peak(torch, dev, stream)
    if args.gather:
        result["gather"] = time_gather(torch, hcdist, b, dev, barrier)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not dry:
        host = host_cpus()
        cores = host["usable"]
        sample = min(args.cpu_sample or 8 * cores, S)
        cb = cpu_baseline(args, cores, [b.encoded(k) for k in range(sample)])
        if cb is not None:
            cb.update(host)
            # the node's physical cores at the measured per-process rate (one stream per process
            # scales linearly until the cores run out; SMT threads beyond them add little)
            cb["node_estimate"] = {"value": cb["value"] / cores * host["physical_cores"], "unit": "GiB/s",
                                   "cores": host["physical_cores"],
                                   "how": "measured value / cores used x the node's physical cores"}
        if cb is not None:
            if not cb["bit_exact_vs_gpu"]:
                raise SystemExit("GPU encodings differ from the reference binary's on the sampled streams")
            result["cpu_baseline"] = cb
            result["bit_exact_vs_reference_streams"] = sample
    del b
    if not dry:
        torch.cuda.empty_cache()
    if world > 1 and not args.no_weak_line:
        result["weak_scaling"] = weak_line(torch, hc, hcdist, args, dev, stream, rank, world, barrier, dry,
                                           use_diff, N)
    cbad = 0
    if not dry and world == 1 and not args.no_configs:
        c5_kernel = S * N / ((enc_ms + dec_ms) * 1e-3) / 2**30 if S == C5_STREAMS and use_diff and \
            args.kind == "photo" else None
        configs, cbad = run_configs(torch, hc, dev, stream, set(), c5_kernel)
        result["configs_bit_exact"] = cbad == 0
        if rank == 0:
            print("detail " + json.dumps({"configs": configs}), flush=True)
        result["configs"] = compact_configs(configs)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    if cbad:
        raise SystemExit(f"config checks FAILED on {cbad} items")
    return result


if __name__ == "__main__":
    main()
