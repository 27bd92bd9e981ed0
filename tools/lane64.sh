#!/bin/bash
# tools/lane64.sh TAG — C2 shard frames with 64 slots per wave and per-lane traces
# (experiment build, XRT_LANE_TRACE) against the default layouts, at N = 1, 8, 32, 128
set -euo pipefail
O=gpurun_out/$1; mkdir -p $O
for n in 1 8 32 128; do
  XRT_LIB=libxrt_hip_exp.so timeout -k 10 200 python3 tools/shard_sim.py C2 --only=$n --timing 2>/dev/null | tail -1 > $O/d$n.json
  XRT_LIB=libxrt_hip_exp.so XRT_LANE_TRACE=1 timeout -k 10 200 python3 tools/shard_sim.py C2 --only=$n --timing --spw=64 2>/dev/null | tail -1 > $O/l$n.json
  python3 -c "
import json
d=json.load(open('$O/d$n.json'))['shards']['$n']['shard_ms']; l=json.load(open('$O/l$n.json'))['shards']['$n']['shard_ms']
print($n, 'default', d, 'lane64', l)"
done
