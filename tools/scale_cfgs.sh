#!/bin/bash
# tools/scale_cfgs.sh TAG [CONFIGS...] — per-shard frame time of shard 0 of N = 1, 2, 4, 8 row
# shards for each config (tools/shard_sim.py): the per-GPU part of an N-GPU strong-scaling run
set -euo pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for c in ${*:-C3 C4 C5}; do
  for n in 1 2 4 8; do
    timeout -k 10 300 python3 tools/shard_sim.py $c --only=$n --timing 2>/dev/null | tail -1 > $O/${c}_$n.json
    python3 -c "import json; d=json.load(open('$O/${c}_$n.json'))['shards']['$n']; print('$c', $n, d['shard_ms'], d['msamples_s'])"
  done
done
