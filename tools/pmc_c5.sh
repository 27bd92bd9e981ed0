#!/bin/bash
# tools/pmc_c5.sh — PMC passes over C5's fused k_step (VolumePathTracing, 64 spp: per-launch
# counters are what matter), one counter group per rocprofv3 run.
set -uo pipefail
O=gpurun_out/pmc_c5; mkdir -p $O; export TMPDIR=/tmp
B=(python3 bench.py --config C5 --spp 64 --steps 1 --warmup 0 --no-cpu --no-timing)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- "${B[@]}" > $O/kt.log 2>&1 && echo kt ok
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/tcc -o tcc --output-format csv -- "${B[@]}" > $O/tcc.log 2>&1 && echo tcc ok
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- "${B[@]}" > $O/fetch.log 2>&1 && echo fetch ok
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY -d $O/sq -o sq --output-format csv -- "${B[@]}" > $O/sq.log 2>&1 && echo sq ok
python3 - <<'PY'
import csv, glob, collections
O = "gpurun_out/pmc_c5"
for tag in ("tcc", "fetch", "sq"):
    f = glob.glob(f"{O}/{tag}/*counter_collection.csv")
    if not f: print(tag, "missing"); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].split("(")[0][-40:]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
    for k, d in acc.items():
        if "k_step" in k or "refill" in k:
            print(tag, k, {c: round(v / max(1, n[(k, c)]), 1) for c, v in d.items()})
PY
grep -E "k_step|k_refill" $O/kt/kt_kernel_stats.csv | cut -c1-160
