#!/bin/bash
# A/B of library builds under the per-file CLI (bench.py configs.C1's workload: hd01.raw -c -m then
# -d, one process per file): median wall and in-process phases per variant, alternating.
#   VARIANTS="noretry nscr" REPS=9 bash scripts/cli_ab.sh
# v = abvar/v/libhcodec.so, loaded through LD_LIBRARY_PATH (the CLI's RUNPATH comes after it).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tmp=$(mktemp -d)
oracle/_ref/huffman-codec-O2 -d -i tests/golden/corpus/hd01.cm.huf -o $tmp/hd01.raw > /dev/null 2>&1 || exit 1
for v in ${VARIANTS:-cur}; do : > gpurun_out/cli_$v.txt; done
for r in $(seq ${REPS:-9}); do
    for v in ${VARIANTS:-cur}; do
        lp=$( [ "$v" = cur ] || echo "abvar/$v")
        for d in "-c -m -i $tmp/hd01.raw -o $tmp/$v.huf" "-d -i $tmp/$v.huf -o $tmp/$v.out"; do
            t0=$(date +%s%N)
            LD_LIBRARY_PATH=$lp HC_CLI_TIMES=1 timeout -k 5 60 huffman-codec_amd/bin/huffman-codec $d 2> $tmp/err || { cat $tmp/err; exit 1; }
            t1=$(date +%s%N)
            echo "${d:0:2} wall_ms=$(( (t1 - t0) / 1000000 )) $(grep hc-times $tmp/err | cut -d' ' -f2-)" >> gpurun_out/cli_$v.txt
        done
        cmp -s $tmp/$v.out $tmp/hd01.raw || { echo "ROUND TRIP FAIL $v"; exit 1; }
    done
done
for v in ${VARIANTS:-cur}; do
    python3 - "$v" <<'PY'
import statistics, sys
v = sys.argv[1]
rows = {"-c": [], "-d": []}
for line in open(f"gpurun_out/cli_{v}.txt"):
    f = line.split()
    rows[f[0]].append({k: float(x) for k, x in (t.split("=") for t in f[1:])})
for d, rs in rows.items():
    print(v, d, " ".join(f"{k} {statistics.median(r[k] for r in rs):.1f}" for k in rs[0]))
PY
done
rm -rf $tmp
