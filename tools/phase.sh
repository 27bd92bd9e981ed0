#!/bin/bash
# tools/phase.sh TAG [N...] — per-phase cycle split of k_step_speculative visits (C2 row shard 0
# of N, default N = 8 and 4) from the XRT_PHASE_CLOCK experiment build:
#   make -C xraytracer_amd/csrc variant TAG=ph DEFS=-DXRT_PHASE_CLOCK=1
# then python3 tools/phase_split.py gpurun_out/TAG
set -euo pipefail
O=gpurun_out/$1; shift; mkdir -p "$O"
for n in ${*:-8 4}; do
  XRT_LIB=${XRT_LIB:-libxrt_hip_ph.so} timeout -k 10 200 python3 tools/shard_sim.py C2 --only=$n --reps=1 --warm-shard \
    > "$O/s$n.out" 2> "$O/s$n.err"
  echo "n=$n $(grep 'phase cycles' "$O/s$n.err" | tail -1)"
done
