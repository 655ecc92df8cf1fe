"""Summarize rocprofv3 PMC passes of scripts/profile.sh: per-kernel counters and per-symbol
instruction counts for the bench workload (8192 photo -m streams: 201635 symbols each)."""
import csv, collections, sys, glob, os
tag = sys.argv[1]
syms = float(sys.argv[2]) if len(sys.argv) > 2 else 8192 * 201635
base = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'gpurun_out', 'prof')
agg = collections.defaultdict(lambda: collections.defaultdict(float))
launches = collections.defaultdict(set)  # per (kernel, pass): dispatches, to report per launch
for f in glob.glob(os.path.join(base, f'{tag}_pmc_*', '*counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        if any(t in k for t in ('encode_kernel<false', 'decode_kernel<false', 'encode_kernel<0', 'decode_kernel<0')):
            kk = 'encode' if 'encode_kernel' in k else 'decode'
            agg[kk][r['Counter_Name']] += float(r['Counter_Value'])
            launches[(kk, r['Counter_Name'])].add(r['Dispatch_Id'])
for k, d in agg.items():
    for c in d:
        d[c] /= max(1, len(launches[(k, c)]))
    cyc = d.get('GRBM_GUI_ACTIVE', 0) / 8
    print(k, f"cycles/XCD {cyc:.3g}")
    for c in ('SQ_INSTS_SALU', 'SQ_INSTS_VALU', 'SQ_INSTS_LDS'):
        if c in d:
            print(f"   {c:16s} per-sym {d[c]/syms:7.2f}   per-CU-cycle {d[c]/256/cyc:.3f}")
    for c in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_VALU', 'SQ_ACTIVE_INST_SCA', 'SQ_ACTIVE_INST_LDS', 'SQ_WAVE_CYCLES', 'SQ_LDS_BANK_CONFLICT'):
        if c in d:
            print(f"   {c:22s} per-sym {d[c]/syms:8.2f}")
