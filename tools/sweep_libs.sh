#!/bin/bash
# tools/sweep_libs.sh CONFIG "LIB..." "V R..." — bench.py throughput for experiment builds
# (csrc/Makefile `variant`) x fused-schedule knobs; one bench process per point.
set -euo pipefail
CFG=$1; LIBS=$2; VRS=$3
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for lib in $LIBS; do
  for vr in $VRS; do
    v=${vr%,*}; r=${vr#*,}
    out=$(XRT_LIB=$lib XRT_STEP_VISITS=$v XRT_STEP_REFILL=$r timeout -k 10 120 python3 "$R/bench.py" --config "$CFG" --steps 2 --warmup 1 --no-cpu 2>/dev/null)
    echo "$lib V=$v R=$r $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], {k: v for k, v in d["roofline"]["kernel_ms_per_step"].items() if v})')"
  done
done
