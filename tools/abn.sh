#!/bin/bash
# tools/abn.sh TAG CONFIG TESTSEL LIB... — GPU tests selected by TESTSEL under each variant LIB,
# then alternating bench frames of CONFIG: the default library and every LIB, two rounds.
set -euo pipefail
O=gpurun_out/$1; C=$2; SEL=$3; shift 3; mkdir -p $O
for lib in "$@"; do
  XRT_LIB=$lib timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -k "$SEL" --timeout 120 --timeout-method thread > $O/tests_$lib.log 2>&1 \
    || { tail -30 $O/tests_$lib.log; exit 1; }
  echo "$lib $(tail -1 $O/tests_$lib.log)"
done
for r in 1 2; do
  for lib in libxrt_hip.so "$@"; do
    XRT_LIB=$lib timeout -k 10 300 python3 bench.py --config $C --steps 3 --warmup 1 --no-cpu > $O/${C}_${lib}_$r.json
    python3 -c "import json; d=json.load(open('$O/${C}_${lib}_$r.json')); print('$C $lib', d['value'], d['ms_per_step'], d['config'].get('iterations_per_frame'))"
  done
done
