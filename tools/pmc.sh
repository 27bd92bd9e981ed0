#!/bin/bash
# tools/pmc.sh TAG CONFIG [bench args] — kernel trace + per-kernel PMC passes of one bench frame
# (SQ timing, SQ instruction mix, TCC hits, FETCH_SIZE, WRITE_SIZE: one counter group per
# rocprofv3 run, MI355X_MICROARCH.md), summarised per kernel by tools/prof_summary.py-style
# averages into gpurun_out/TAG/summary.txt.  E.g. tools/pmc.sh c4 C4 --spp 64
set -uo pipefail
TAG=$1; CFG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG; mkdir -p "$O"; export TMPDIR=/tmp
B=(python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 0 --no-cpu --no-timing "$@")
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- "${B[@]}" > "$O/kt.log" 2>&1 && echo kt ok
run() { local t=$1; shift; timeout -s KILL 200 rocprofv3 --pmc "$@" -d "$O/$t" -o "$t" --output-format csv -- "${B[@]}" > "$O/$t.log" 2>&1 && echo "$t ok"; }
run sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU \
    SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS
run sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM
run tcc TCC_HIT_sum TCC_MISS_sum
run fetch FETCH_SIZE
run write WRITE_SIZE
python3 - "$O" > "$O/summary.txt" <<'PY'
import collections, csv, glob, re, sys
O = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for t in ("sq1", "sq2", "tcc", "fetch", "write"):
    for f in glob.glob(f"{O}/{t}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_\w+)", r["Kernel_Name"])
            k = m.group(1) if m else r["Kernel_Name"][:40]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
for f in glob.glob(f"{O}/kt/**/*kernel_stats.csv", recursive=True):
    for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:8]:
        print(f'{float(r["TotalDurationNs"])/1e6:10.1f} ms {int(r["Calls"]):7d} calls {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:100]}')
for k, c in acc.items():
    per = {name: v / max(1, n[(k, name)]) for name, v in c.items()}   # per dispatch
    line = f"{k}: " + " ".join(f"{name}={v:.4g}" for name, v in sorted(per.items()))
    if c.get("SQ_WAVE_CYCLES"):
        line += (f" | lane_util {c['SQ_THREAD_CYCLES_VALU'] / max(1, 64 * c['SQ_ACTIVE_INST_VALU']):.3f}"
                 f" wait {c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.3f} valu {c['SQ_ACTIVE_INST_VALU'] / c['SQ_WAVE_CYCLES']:.3f}")
    print(line)
PY
cat "$O/summary.txt"
