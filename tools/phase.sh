#!/bin/bash
# tools/phase.sh TAG — per-phase cycle split of k_step_merged for C2 at 1, 8 and 128 row
# shards, from the XRT_PHASE_CLOCK experiment build:
#   make -C xraytracer_amd/csrc variant TAG=ph DEFS=-DXRT_PHASE_CLOCK
set -euo pipefail
O=gpurun_out/$1; mkdir -p $O
for n in 1 8 128; do
  XRT_LIB=${XRT_LIB:-libxrt_hip_ph.so} timeout -k 10 200 python3 tools/shard_sim.py C2 --only=$n --timing > $O/s$n.out 2> $O/s$n.err
  echo "n=$n $(tail -1 $O/s$n.out)"
  grep "phase cycles" $O/s$n.err | tail -1
done
