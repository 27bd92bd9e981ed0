#!/bin/bash
# tools/ab_cfg.sh TAG LIB_A LIB_B CONFIG... — bench.py frame time of each config under two libraries
set -euo pipefail
O=gpurun_out/$1; mkdir -p $O; A=$2; B=$3; shift 3
for c in "$@"; do
  for lib in $A $B; do
    XRT_LIB=$lib timeout -k 10 300 python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu > $O/${c}_$lib.json
    python3 -c "import json; d=json.load(open('$O/${c}_$lib.json')); print('$c', '$lib', d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms_per_step'))"
  done
done
