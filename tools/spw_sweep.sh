#!/bin/bash
# tools/spw_sweep.sh TAG — C2 per-shard frame time for each slots-per-wave layout of the
# merged kernel (16/32/64 slots per wave, group traces on/off) at 1 ... 32 row shards
set -euo pipefail
O=gpurun_out/$1; mkdir -p $O
for n in 1 2 4 8 16 32; do
  for v in "--spw=64" "--spw=32" "--spw=32 --no-group" "--spw=16" "--spw=16 --no-group"; do
    timeout -k 10 200 python3 tools/shard_sim.py C2 --only=$n $v 2>/dev/null | tail -1 > $O/tmp.json
    python3 -c "import json; d=json.load(open('$O/tmp.json'))['shards']['$n']; print($n, '$v', d['shard_ms'])"
  done
done
