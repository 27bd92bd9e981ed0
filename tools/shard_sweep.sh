#!/bin/bash
# tools/shard_sweep.sh [N] — shard 0 of N (C2) under each merged-schedule layout
# (slots per wave x group trace), plus a phase-clock build for the default layout.
set -euo pipefail
N=${1:-8}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out/sweep"
run() { echo "== $*"; env "$@" timeout -k 10 120 python3 "$R/tools/shard_sim.py" C2 --only=$N --timing 2>&1 | grep -v amdgpu.ids | head -2; }
run XRT_MERGED_SPW=64
run XRT_MERGED_SPW=32
run XRT_MERGED_SPW=16
run XRT_MERGED_SPW=32 XRT_NO_GROUP=1
run XRT_MERGED_SPW=16 XRT_NO_GROUP=1
run XRT_MERGED_SPW=64 XRT_LANE_TRACE=1
run XRT_LIB=libxrt_hip_ph.so XRT_MERGED_SPW=16
run XRT_LIB=libxrt_hip_ph.so XRT_MERGED_SPW=64
