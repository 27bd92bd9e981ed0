#!/bin/bash
# tools/ab_c4.sh TAG LIB... — C4 bench (256 spp) per experiment library, interleaved twice
set -euo pipefail
O=gpurun_out/$1; shift; mkdir -p $O
for rep in 1 2; do
  for lib in "$@"; do
    XRT_LIB=$lib timeout -k 10 200 python3 bench.py --config C4 --spp 256 --steps 2 --warmup 1 --no-cpu > $O/b_${lib}_$rep.json
    python3 -c "
import json; b=json.load(open('$O/b_${lib}_$rep.json')); print('$lib', $rep, b['value'], b['ms_per_step'], b['roofline'].get('kernel_ms_per_step'))"
  done
done
