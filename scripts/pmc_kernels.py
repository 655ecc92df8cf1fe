"""Per-kernel PMC table from one rocprofv3 --pmc pass (diagnostic):

    python scripts/pmc_kernels.py gpurun_out/prof/pmcX [kernel-substring ...]

Counters are summed over the dimensions rocprofv3 reports per dispatch, then averaged over the
kernel's dispatches; per-wave values divide by SQ_WAVES of the same dispatch."""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    want = sys.argv[2:]
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, dispatch) -> counters
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if want and not any(w in k for w in want):
                continue
            per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for (k, _), c in per.items():
        n[k] += 1
        for name, v in c.items():
            agg[k][name] += v
    for k in sorted(agg):
        c = {name: v / n[k] for name, v in agg[k].items()}
        waves = c.get("SQ_WAVES", 0) or 1
        short = k.replace("hc::(anonymous namespace)::", "").split("(")[0][:40]
        cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
        fields = " ".join(f"{name.replace('SQ_', '').lower()}={v / waves:.0f}" for name, v in sorted(c.items())
                          if name not in ("SQ_WAVES", "GRBM_GUI_ACTIVE"))
        print(f"{short:40s} n={n[k]} waves={waves:.0f} cycles/XCD={cyc:.3g} per-wave: {fields}")


if __name__ == "__main__":
    main()
