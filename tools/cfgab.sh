#!/bin/bash
# tools/cfgab.sh TAG CONFIG LIB... — one bench frame of CONFIG per library
set -euo pipefail
O=gpurun_out/$1; CFG=$2; shift 2; mkdir -p $O
for lib in "$@"; do
  XRT_LIB=$lib timeout -k 10 300 python3 bench.py --config $CFG --steps 1 --warmup 1 --no-cpu > $O/${CFG}_$lib.json
  python3 -c "import json; d=json.load(open('$O/${CFG}_$lib.json')); print('$CFG', '$lib', d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms_per_step'))"
done
