"""Per-kernel launch durations from a rocprofv3 kernel trace, grouped by kernel and grid size
(each config of a bench run launches with its own grid), library kernels only.

    python scripts/trace_summary.py gpurun_out/prof/<run>/<name>_kernel_trace.csv
"""
import collections
import csv
import re
import sys


def short(name):
    m = re.search(r"(\w+_kernel)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def main(path):
    agg = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if "at::" in n or "rocclr" in n:
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        key = (short(n), r["Grid_Size_X"])
        agg.setdefault(key, []).append(d)
    for (k, g), ds in agg.items():
        print(f"{k:34s} grid {g:>9s}  n {len(ds):3d}  avg {sum(ds) / len(ds):10.4f} ms  min {min(ds):10.4f}")


if __name__ == "__main__":
    main(sys.argv[1])
