"""One line per config of a bench.py JSON line (the headline, then `configs`):
    python3 scripts/bench_summary.py gpurun_out/<tag>_bench.log"""
import json
import sys

for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    r = json.loads(line)
    if "value" in r:
        cb = (r.get("cpu_baseline") or {}).get("value")
        print("C5", r["value"], "GiB/s enc", r["encode_ms"], "dec", r["decode_ms"], "frac", r["roofline"]["frac"],
              "cpu", cb)
    for k, v in r.get("configs", {}).items():
        if k == "C1":
            print("C1", {b: (x["encode_s"], x["decode_s"], x["encode_bytes_identical_to_reference"])
                         for b, x in v.get("binaries", {}).items()})
            continue
        print(k, v.get("encode_ms"), v.get("decode_ms"), v.get("GiBps"), v.get("round_trip_exact"),
              v.get("reference_digests_identical"))
        for d in ("encode", "decode"):
            st = (v.get("stages") or {}).get(d)
            if st:
                print("   ", d, {s: x["ms"] for s, x in st.items() if x.get("ms", 0) > 0.05})
