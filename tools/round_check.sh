#!/bin/bash
# tools/round_check.sh TAG — after a host-side change: GPU tests, the default bench line,
# and the C2 shard table (tools/shard_table.sh) on one box.
set -euo pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; tail -1 $O/gpu_tests.log
timeout -k 10 300 python3 bench.py --no-cpu > $O/bench.json; cut -c1-220 $O/bench.json
tools/shard_table.sh $1_shards
