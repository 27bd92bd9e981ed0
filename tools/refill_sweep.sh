#!/bin/bash
# tools/refill_sweep.sh TAG — C2 bench at several refill grid sizes (XRT_REFILL_BLOCKS)
set -euo pipefail
O=gpurun_out/$1; mkdir -p $O
for B in 2048 4096 8192 16384; do
  XRT_REFILL_BLOCKS=$B timeout -k 10 200 python3 bench.py --config C2 --steps 3 --warmup 1 --no-cpu > $O/b$B.json
  python3 -c "import json; d=json.load(open('$O/b$B.json')); print($B, d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])"
done
