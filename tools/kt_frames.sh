#!/bin/bash
# tools/kt_frames.sh TAG CONFIG [bench args] — per-launch k_step durations over several frames
set -euo pipefail
TAG=$1; CFG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/kt" -o kt --output-format csv -- \
    python3 "$R/bench.py" --config "$CFG" --no-cpu --no-timing "$@" > "$OUT/kt.log" 2>&1
python3 - "$OUT/kt" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
line = []
for r in rows:
    n = r["Kernel_Name"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if "k_seed" in n:
        if line: print(" ".join(line))
        line = [f"@{(int(r['Start_Timestamp'])-t0)/1e6:.1f}ms:"]
    if "k_step" in n or "k_trace" in n or "k_shade" in n:
        line.append(f"{d:.0f}")
print(" ".join(line))
PY
