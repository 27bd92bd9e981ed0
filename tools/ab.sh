#!/bin/bash
# tools/ab.sh TAG LIB — C2 1-GPU bench and 8/128-shard frames, default library vs experiment LIB
set -euo pipefail
O=gpurun_out/$1; mkdir -p $O
for lib in libxrt_hip.so $2; do
  XRT_LIB=$lib timeout -k 10 200 python3 bench.py --config C2 --steps 2 --warmup 1 --no-cpu > $O/b_$lib.json
  for n in 8 128; do
    XRT_LIB=$lib timeout -k 10 200 python3 tools/shard_sim.py C2 --only=$n --timing 2>/dev/null | tail -1 > $O/s${n}_$lib.json
  done
  python3 -c "
import json; b=json.load(open('$O/b_$lib.json'))
s8=json.load(open('$O/s8_$lib.json'))['shards']['8']['shard_ms']; s128=json.load(open('$O/s128_$lib.json'))['shards']['128']['shard_ms']
print('$lib', b['value'], b['ms_per_step'], 'shard8', s8, 'shard128', s128)"
done
