#!/bin/bash
# tools/shard_ab.sh TAG LIB... — C2 per-shard frame time at 1, 8, 32 and 128 row shards per library
set -euo pipefail
O=gpurun_out/$1; shift; mkdir -p $O
for lib in "$@"; do
  for n in 1 8 32 128; do
    XRT_LIB=$lib timeout -k 10 200 python3 tools/shard_sim.py C2 --only=$n 2>/dev/null | tail -1 > $O/s${n}_$lib.json
  done
  python3 -c "
import json
print('$lib', [json.load(open('$O/s%d_$lib.json' % n))['shards'][str(n)]['shard_ms'][0] for n in (1, 8, 32, 128)])"
done
