#!/bin/bash
# tools/phase_ab.sh TAG LIB... — per-phase cycles and pair-pass counts of k_step_merged (C2,
# 1 and 8 row shards) for each -DXRT_PHASE_CLOCK experiment library
set -euo pipefail
O=gpurun_out/$1; shift; mkdir -p $O
for lib in "$@"; do
  for n in 1 8; do
    XRT_LIB=$lib timeout -k 10 200 python3 tools/shard_sim.py C2 --only=$n --timing > $O/${lib}_$n.out 2> $O/${lib}_$n.err
    echo "$lib n=$n $(tail -1 $O/${lib}_$n.out | cut -c1-120)"
    grep "phase cycles" $O/${lib}_$n.err | tail -1
  done
done
