#!/bin/bash
# tools/evidence.sh TAG [CONFIG] — the measurement evidence of a round, on the GPU box:
#   1. rocprofv3 kernel-trace/stats + PMC passes of bench.py (tools/profile.sh)
#   2. per-launch HBM traffic / SQ counters of the dominant kernel -> profiles/{traffic,pmc}_CONFIG.json
#   3. the default bench.py line (with the CPU baseline) -> gpurun_out/TAG/bench.json
# Copy gpurun_out/TAG/{kt_kernel_stats.csv,summary.txt,bench.json} into profiles/ after.
set -euo pipefail
TAG=$1; CFG=${2:-C2}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
"$R/tools/profile.sh" "$CFG" "$TAG"
KPAT=$(python3 - "$R/gpurun_out/$TAG/kt" <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/*kernel_stats.csv")[0])))
top = max(rows, key=lambda r: float(r["TotalDurationNs"]))
import re
k = re.search(r"(k_\w+)", top["Name"]).group(1)
# the merged schedule's step launches (xrt_stats' XRT_K_STEP family) include the speculative kernel
print("k_step_merged|k_step_spec" if k == "k_step_merged" else k)
PY
)
python3 "$R/tools/prof_summary.py" "$R/gpurun_out/$TAG" "$KPAT" --traffic "$CFG" "$R/profiles/traffic_$CFG.json" \
    --pmc "$CFG" "$R/profiles/pmc_$CFG.json" --csv "$R/gpurun_out/$TAG/pmc_dispatch.csv" > "$R/gpurun_out/$TAG/summary.txt"
cp "$R/gpurun_out/$TAG/kt/kt_kernel_stats.csv" "$R/gpurun_out/$TAG/kt_kernel_stats.csv"
# raw rocprofv3 output (every dispatch of every pass) can exceed gpurun's 64 MiB copy-back:
# keep the summaries and the gzipped per-dispatch counters of the dominant kernel only
gzip -f "$R/gpurun_out/$TAG/pmc_dispatch.csv"
rm -rf "$R/gpurun_out/$TAG"/{kt,sq1,sq2,fetch,write}
mkdir -p "$R/gpurun_out/profiles_new" && cp "$R/profiles/traffic_$CFG.json" "$R/profiles/pmc_$CFG.json" "$R/gpurun_out/profiles_new/"
timeout -k 10 600 python3 "$R/bench.py" --config "$CFG" > "$R/gpurun_out/$TAG/bench.json"
cat "$R/gpurun_out/$TAG/bench.json"
