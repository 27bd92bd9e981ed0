#!/bin/bash
# tools/shards.sh TAG [pytest -k expr] — GPU parity subset, then the C2 per-shard frame time at
# 2, 4, 8 and 128 row shards (tools/shard_sim.py)
set -euo pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${2:-shards or slots or merged or cornell or c1}" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for n in 2 4 8 128; do
  timeout -k 10 200 python3 tools/shard_sim.py C2 --only=$n --timing 2>/dev/null | tail -1 > $O/s$n.json
  python3 -c "import json; d=json.load(open('$O/s$n.json'))['shards']['$n']; print($n, d['shard_ms'], d['kernel_ms'].get('step'))"
done
