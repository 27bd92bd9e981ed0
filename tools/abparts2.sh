#!/bin/bash
set -euo pipefail
O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for lib in libxrt_hip.so "$@"; do
  r=""
  for c in "C4 --spp=256 --only=1" "C4 --only=8" "C2 --only=1" "C2 --only=8" "C3 --only=1" "C5 --only=1"; do
    set -- $c
    n=${!#}; n=${n#--only=}
    XRT_LIB=$lib timeout -k 10 300 python3 tools/shard_sim.py $c --timing 2>/dev/null | tail -1 > $O/s.json
    r="$r $1/$n: $(python3 -c "import json; print(json.load(open('$O/s.json'))['shards']['$n']['shard_ms'][0])")"
  done
  echo "$lib $r"
done
