#!/bin/bash
# tools/costmap.sh TAG LIB... — timing-only cost map of the C2 merged kernel: for the default
# library and each experiment build LIB (csrc/Makefile `variant`, e.g. -DXRT_EXP_FASTDIV:
# inexact math, so images differ; paths stay statistically alike), the 1-GPU frame and the
# 8- and 128-shard frames.  The time a switch removes bounds what that piece costs.
set -euo pipefail
O=gpurun_out/$1; shift; mkdir -p $O
for lib in libxrt_hip.so "$@"; do
  for n in 1 8 128; do
    XRT_LIB=$lib timeout -k 10 200 python3 tools/shard_sim.py C2 --only=$n --timing 2>/dev/null | tail -1 > $O/s${n}_$lib.json
  done
  python3 -c "
import json
r = [json.load(open('$O/s%d_$lib.json' % n))['shards'][str(n)]['shard_ms'][0] for n in (1, 8, 128)]
print('$lib'.ljust(28), 'shard ms  1: %.2f  8: %.2f  128: %.2f' % tuple(r))"
done
