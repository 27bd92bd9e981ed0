#!/bin/bash
# tools/cfg_lines.sh TAG — smoke, the GPU parity suite and the C3 / C4 / C5 bench lines
set -euo pipefail
TAG=${1:-cfg}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; tail -1 $O/smoke.log
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; tail -1 $O/gpu_tests.log
for c in C3 C4 C5; do
  timeout -k 10 300 python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu > $O/bench_$c.json
  python3 -c "import json; d=json.load(open('$O/bench_$c.json')); print('$c', d['value'], d['ms_per_step'])"
done
