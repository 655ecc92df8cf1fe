"""Turn a scripts/profile.sh run (gpurun_out/prof/<tag>_*) into the committed evidence:

  profiles/<round>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (as written)
  profiles/<round>_pmc_summary.json   per-launch PMC counters of the FGK kernels + per-symbol rates
  profiles/pmc_summary.json           what bench.py reads for roofline.traffic and issue: per
                                      launch HBM bytes and VALU + SALU instructions, keyed
                                      kernel:mode:kind:streams, stamped with the sha of
                                      hc_fgk.hip (bench.py ignores it once the source changes)

    python scripts/profile_artifacts.py <tag> <round> [--streams S] [--mode cm] [--kind photo]

HBM bytes = FETCH_SIZE x 2 + WRITE_SIZE (KB -> B). The x2: on gfx950 FETCH_SIZE counts half of
wide streaming reads (MI355X_MICROARCH.md, HBM / rocprofv3); the kernels' loads are 4 B/lane,
which the guide lists as uncalibrated, so the factor is checked against a known byte count: the
encoder reads exactly streams x 262144 raw bytes, and x2 FETCH_SIZE reproduces that (the check
is printed: `encoder_read_check`).
"""
import argparse
import collections
import csv
import glob
import hashlib
import json
import os
import re
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FGK_SRC = os.path.join(ROOT, "huffman-codec_amd", "csrc", "hc_fgk.hip")


def kernel_key(name):
    """encode_kernel<0, 1, false> (tree layout 0 = narrow, source 1, path-cache mode; round-1 builds:
    <false, 1>) -> ('encode_kernel', narrow, source / destination kind). The table-mode launch of
    the same layout (<0, 1, true>) and the small-alphabet launches (encode_kernel<0, 1, false, true>,
    decode_kernel<0, 0, true>) are keyed apart (_tables, _small): each stream is coded by one
    of them, so a workload's total is their sum."""
    m = re.search(r"(encode_kernel|decode_kernel)<(false|true|\d), (\d)((?:, (?:false|true))*)>", name)
    if not m:
        return None
    flags = [f.strip() == "true" for f in m.group(4).split(",")[1:]]
    # encode_kernel<layout, source, kTab, kSmall>, decode_kernel<layout, destination, kSmall>
    tab = m.group(1) == "encode_kernel" and len(flags) > 0 and flags[0]
    small = flags[-1] if (m.group(1) == "encode_kernel" and len(flags) > 1) or (m.group(1) == "decode_kernel" and flags) else False
    name = m.group(1) + ("_tables" if tab else "") + ("_small" if small else "")
    return (name, m.group(2) in ("false", "0"), int(m.group(3)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("round")
    ap.add_argument("--streams", type=int, default=65536)
    ap.add_argument("--mode", default="cm")
    ap.add_argument("--kind", default="photo")
    ap.add_argument("--symbols", type=float, default=0.0,
                    help="FGK symbols per stream (default: fgk_symbols_per_stream of the stats pass's bench line)")
    a = ap.parse_args()
    if not a.symbols:
        log = os.path.join(ROOT, "gpurun_out", "prof", f"{a.tag}_stats.log")
        for line in open(log):
            if line.startswith("{"):
                a.symbols = float(json.loads(line)["fgk_symbols_per_stream"])
        if not a.symbols:
            raise SystemExit(f"no fgk_symbols_per_stream in {log}: pass --symbols")
    prof = os.path.join(ROOT, "gpurun_out", "prof")
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = glob.glob(os.path.join(prof, f"{a.tag}_stats", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(out, f"{a.round}_kernel_stats.csv"))

    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.defaultdict(set)
    for f in glob.glob(os.path.join(prof, f"{a.tag}_pmc_*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = kernel_key(r["Kernel_Name"])
            if not k or not k[1]:  # the narrow variants code the photo streams; the wide ones exit
                continue
            name = k[0]
            agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
            launches[(name, r["Counter_Name"])].add(r["Dispatch_Id"])
    syms = a.symbols * a.streams
    src = hashlib.sha256(open(FGK_SRC, "rb").read()).hexdigest()[:16]
    summary = {"workload": f"bench.py --streams {a.streams} ({a.kind} -{a.mode.replace('m', ' -m')}, 512x512); "
                           "counters per launch", "source_sha": src, "symbols_per_launch": syms,
               "note": "rocprofv3 --pmc passes, one counter group per run (never combined with tracing); "
                       "FETCH_SIZE / WRITE_SIZE in KB as reported",
               "counters": {}, "per_symbol": {}, "hbm_bytes_per_launch": {}}
    bench = {"source_sha": src, "launches": {},
             "_note": f"per-launch HBM bytes (FETCH_SIZE x2 + WRITE_SIZE) and SQ_INSTS_VALU + SQ_INSTS_SALU from "
                      f"rocprofv3 PMC passes; details in profiles/{a.round}_pmc_summary.json"}
    for name, d in agg.items():
        per = {c: v / max(1, len(launches[(name, c)])) for c, v in d.items()}
        summary["counters"][name] = per
        summary["per_symbol"][name] = {c: round(per[c] / syms, 3) for c in per
                                       if c.startswith("SQ_INSTS") or c.startswith("SQ_ACTIVE") or
                                       c.startswith("SQ_WAIT") or c == "SQ_WAVE_CYCLES"}
        e = {}
        if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
            b = int(round((per["FETCH_SIZE"] * 2 + per["WRITE_SIZE"]) * 1024))
            summary["hbm_bytes_per_launch"][name] = b
            e["hbm_bytes"] = b
            if name == "encode_kernel":
                summary["encoder_read_check"] = {"fetch_x2_bytes": per["FETCH_SIZE"] * 2 * 1024,
                                                 "raw_bytes": a.streams * 262144.0}
        if "SQ_INSTS_VALU" in per and "SQ_INSTS_SALU" in per:
            e["valu_salu_insts"] = per["SQ_INSTS_VALU"] + per["SQ_INSTS_SALU"]
        bench["launches"][f"{name}:{a.mode}:{a.kind}:{a.streams}"] = e
    with open(os.path.join(out, f"{a.round}_pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    # other workloads' entries measured on the same source stay (one file, keyed per workload)
    path = os.path.join(out, "pmc_summary.json")
    if os.path.exists(path):
        old = json.load(open(path))
        if old.get("source_sha") == src:
            for k, v in old.get("launches", {}).items():
                bench["launches"].setdefault(k, v)
    bench["_note"] = ("per-launch HBM bytes (FETCH_SIZE x2 + WRITE_SIZE) and SQ_INSTS_VALU + SQ_INSTS_SALU from "
                      "rocprofv3 PMC passes, keyed kernel:mode:kind:streams; details in profiles/r*_pmc_summary.json")
    with open(path, "w") as f:
        json.dump(bench, f, indent=1)
    print(json.dumps(summary["per_symbol"], indent=1))
    print(json.dumps(bench, indent=1))
    print(json.dumps(summary.get("encoder_read_check"), indent=1))


if __name__ == "__main__":
    main()
