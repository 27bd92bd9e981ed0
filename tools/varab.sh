#!/bin/bash
# tools/varab.sh TAG LIB TESTSEL CONFIG... — GPU parity tests selected by TESTSEL (pytest -k) under
# the experiment library LIB, then one bench frame and the 8-shard frame of each CONFIG under the
# default library and LIB.  Stops at the first failing step.
set -euo pipefail
O=gpurun_out/$1; LIB=$2; SEL=$3; shift 3; mkdir -p $O
XRT_LIB=$LIB timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -k "$SEL" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in "$@"; do
  for lib in libxrt_hip.so $LIB; do
    XRT_LIB=$lib timeout -k 10 300 python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu > $O/${c}_$lib.json
    XRT_LIB=$lib timeout -k 10 200 python3 tools/shard_sim.py $c --only=8 --timing 2>/dev/null | tail -1 > $O/${c}_s8_$lib.json
    python3 -c "
import json; d=json.load(open('$O/${c}_$lib.json')); s=json.load(open('$O/${c}_s8_$lib.json'))['shards']['8']
print('$c', '$lib', d['value'], d['ms_per_step'], 'shard8', s['shard_ms'], s['kernel_ms'])"
  done
done
