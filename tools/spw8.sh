#!/bin/bash
# tools/spw8.sh TAG — C2 shard frame at N = 8 and 128 for each merged-kernel layout
set -euo pipefail
O=gpurun_out/$1; mkdir -p $O
for n in 8 128; do
  for v in "--spw=64" "--spw=32" "--spw=32 --no-group" "--spw=16" "--spw=16 --no-group" "--spw=4"; do
    timeout -k 10 200 python3 tools/shard_sim.py C2 --only=$n --timing $v 2>/dev/null | tail -1 > $O/tmp.json
    python3 -c "import json; d=json.load(open('$O/tmp.json'))['shards']['$n']; print($n, '$v', d['shard_ms'], d['iterations'])"
  done
done
