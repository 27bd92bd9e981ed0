#!/bin/bash
# tools/c4ab.sh TAG LIB... — C4 bench line (1 frame) per library
set -euo pipefail
O=gpurun_out/$1; shift; mkdir -p $O
for lib in "$@"; do
  XRT_LIB=$lib timeout -k 10 300 python3 bench.py --config C4 --steps 1 --warmup 1 --no-cpu > $O/c4_$lib.json
  python3 -c "import json; d=json.load(open('$O/c4_$lib.json')); print('C4', '$lib', d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms_per_step'))"
done
