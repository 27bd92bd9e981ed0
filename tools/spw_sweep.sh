#!/bin/bash
# tools/spw_sweep.sh TAG — C2 per-shard frame at 2 and 4 shards under each slots-per-wave layout
set -euo pipefail
O=gpurun_out/$1; mkdir -p $O
for n in 2 4; do
  for spw in 64 32 16; do
    XRT_MERGED_SPW=$spw timeout -k 10 200 python3 tools/shard_sim.py C2 --only=$n --timing 2>/dev/null | tail -1 > $O/s${n}_$spw.json
    python3 -c "import json; d=json.load(open('$O/s${n}_$spw.json'))['shards']['$n']; print($n, $spw, d['shard_ms'], d['kernel_ms'].get('step'))"
  done
done
