#!/bin/bash
# tools/quick.sh TAG [pytest -k expr] — GPU parity tests (subset), C2 bench line, 8-shard C2 time
set -euo pipefail
TAG=${1:-quick}; K=${2:-}
O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
else
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
fi
tail -1 $O/t.log
timeout -k 10 200 python3 bench.py --config C2 --steps 3 --warmup 1 --no-cpu > $O/b.json
python3 -c "import json; d=json.load(open('$O/b.json')); print('C2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])"
timeout -k 10 200 python3 tools/shard_sim.py C2 --only=8 --timing 2>/dev/null | tail -1 > $O/s8.json
cat $O/s8.json
