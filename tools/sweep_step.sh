#!/bin/bash
# tools/sweep_step.sh [CONFIG] — C2 (default) throughput over the fused-schedule knobs
# XRT_STEP_VISITS x XRT_STEP_REFILL; one bench.py process per point, each under a timeout.
set -euo pipefail
CFG=${1:-C2}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out"
for vr in "4 2" "4 4" "8 1" "8 2" "2 4" "16 1" "6 2"; do
    set -- $vr
    out=$(XRT_STEP_VISITS=$1 XRT_STEP_REFILL=$2 timeout -k 10 120 python3 "$R/bench.py" --config "$CFG" --steps 2 --warmup 1 --no-cpu 2>/dev/null)
    echo "V=$1 R=$2 $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms_per_step"])')"
done
