#!/bin/bash
set -uo pipefail
for lib in libxrt_hip.so libxrt_hip_w3.so libxrt_hip_w2.so; do
  for n in 1 8; do
    echo "lib=$lib n=$n $(XRT_LIB=$lib timeout -k 10 100 python3 tools/shard_sim.py C2 --only=$n --timing 2>/dev/null | head -1)"
  done
done
