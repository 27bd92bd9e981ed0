#!/bin/bash
# tools/shard_table.sh TAG — C2 per-shard frame time for N = 1 ... 128 row shards
set -euo pipefail
O=gpurun_out/$1; mkdir -p $O
for n in 1 2 4 8 16 32 64 128; do
  timeout -k 10 200 python3 tools/shard_sim.py C2 --only=$n --timing 2>/dev/null | tail -1 > $O/s$n.json
  python3 -c "import json; d=json.load(open('$O/s$n.json'))['shards']['$n']; print($n, d['shard_ms'], d['kernel_ms'])"
done
