#!/bin/bash
# tools/kt_quick.sh TAG CONFIG [bench args] — rocprofv3 kernel stats + SQ timing PMC of one bench frame
set -euo pipefail
TAG=$1; CFG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
B=(python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 0 --no-cpu --no-timing "$@")
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- "${B[@]}" > "$OUT/kt.log" 2>&1
python3 - "$OUT/kt" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(f'{float(r["TotalDurationNs"])/1e6:10.1f} ms {int(r["Calls"]):7d} calls {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:90]}')
PY
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS \
    -d "$OUT/sq1" -o sq1 --output-format csv -- "${B[@]}" > "$OUT/sq1.log" 2>&1
python3 - "$OUT/sq1" <<'PY'
import csv, glob, sys, re, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    m = re.search(r"(k_\w+)", r["Kernel_Name"])
    if not m: continue
    k = m.group(1)
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in acc.items():
    if c["SQ_WAVE_CYCLES"] == 0: continue
    lu = c["SQ_THREAD_CYCLES_VALU"] / max(1, 64 * c["SQ_ACTIVE_INST_VALU"])
    print(f'{k:18s} lane_util {lu:.3f} wait {c["SQ_WAIT_ANY"]/c["SQ_WAVE_CYCLES"]:.2f} issue_stall {c["SQ_WAIT_INST_ANY"]/c["SQ_WAVE_CYCLES"]:.2f} active {c["SQ_ACTIVE_INST_ANY"]/c["SQ_WAVE_CYCLES"]:.2f} valu {c["SQ_ACTIVE_INST_VALU"]/c["SQ_WAVE_CYCLES"]:.2f}')
PY
