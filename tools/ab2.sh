#!/bin/bash
# tools/ab2.sh TAG LIB CONFIG [REPS] — the full GPU suite under the default library, then
# alternating default / LIB bench frames of CONFIG (REPS pairs), one JSON summary line each.
set -euo pipefail
O=gpurun_out/$1; LIB=$2; C=$3; N=${4:-2}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for r in $(seq $N); do
  for lib in libxrt_hip.so $LIB; do
    XRT_LIB=$lib timeout -k 10 300 python3 bench.py --config $C --steps 3 --warmup 1 --no-cpu > $O/${C}_${lib}_$r.json
    python3 -c "import json; d=json.load(open('$O/${C}_${lib}_$r.json')); print('$C $lib', d['value'], d['ms_per_step'], d['config'].get('iterations_per_frame'))"
  done
done
