#!/bin/bash
# tools/trace2.sh — trace cost per visit: the default build vs a build that traces twice
set -uo pipefail
for n in 8 128; do
  for lib in libxrt_hip.so libxrt_hip_t2.so; do
    for spw in 16 64; do
      echo "n=$n lib=$lib spw=$spw $(XRT_LIB=$lib XRT_MERGED_SPW=$spw timeout -k 10 100 python3 tools/shard_sim.py C2 --only=$n --timing 2>/dev/null | head -1)"
    done
  done
done
