"""Per-kernel, per-wave PMC rates from a rocprofv3 --pmc run (counter_collection.csv), grouped
by kernel name; `last` = only the last N dispatches of each kernel (one config's launches).

    python scripts/pmc_table.py gpurun_out/prof/<tag>/pmc_counter_collection.csv [last]
"""
import collections
import csv
import re
import sys


def main(path, last=0):
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    for r in csv.DictReader(open(path)):
        m = re.search(r"(\w+_kernel)(<[^>]*>)?", r["Kernel_Name"])
        if not m or "at::" in r["Kernel_Name"]:
            continue
        k = m.group(1) + (m.group(2) or "")
        d = per[k][int(r["Dispatch_Id"])]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k, disp in per.items():
        ids = sorted(disp)[-last:] if last else sorted(disp)
        tot = collections.defaultdict(float)
        for i in ids:
            for c, v in disp[i].items():
                tot[c] += v
        n = len(ids)
        waves = tot.get("SQ_WAVES", 0) / n or 1
        row = {c: v / n / (waves if c.startswith("SQ_INSTS") or c in ("SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY") else 1)
               for c, v in tot.items()}
        print(f"{k:30s} n={n} ms={row['_ns'] / 1e6:.3f} waves={waves:.0f} " +
              " ".join(f"{c.replace('SQ_', '').lower()}={v:.0f}" for c, v in sorted(row.items())
                       if c not in ("_ns", "SQ_WAVES")))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0)
