#!/bin/bash
# tools/quick2.sh TAG [pytest -k expr] — GPU parity subset, then C2 shard frames at N = 1, 8, 128
# (default layouts) and 128 at 16 slots per wave (a 4-lane group alone on its SIMD)
set -euo pipefail
TAG=$1; K=${2:-"merged or group or shard or headline"}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $O/t.log 2>&1 \
  || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for a in "1" "8" "128" "128 --spw=16"; do
  set -- $a
  timeout -k 10 200 python3 tools/shard_sim.py C2 --only=$1 --timing ${2:-} 2>/dev/null | tail -1 > $O/s.json
  python3 -c "import json; d=json.load(open('$O/s.json'))['shards']['$1']; print('shards $a', d['shard_ms'], d['kernel_ms'].get('step'))"
done
