#!/bin/bash
# tools/launches.sh TAG [CONFIG] — per-launch kernel times and live hints (experiment build,
# XRT_TRACE_LAUNCHES) of shard 0 of N = 1 and 8
set -euo pipefail
O=gpurun_out/$1; C=${2:-C2}; mkdir -p $O
for n in 1 8; do
  XRT_LIB=libxrt_hip_exp.so XRT_TRACE_LAUNCHES=1 timeout -k 10 300 python3 tools/shard_sim.py $C --only=$n --timing \
    > $O/s$n.out 2> $O/s$n.err
  tail -1 $O/s$n.out | cut -c1-200
done
