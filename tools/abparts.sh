#!/bin/bash
# tools/abparts.sh TAG LIB — default library vs LIB: C4 (256 spp, one GPU and shard 0 of 8)
# and C2 (one GPU and shard 0 of 8) frame times
set -euo pipefail
O=gpurun_out/$1; mkdir -p $O
for lib in libxrt_hip.so $2 libxrt_hip.so $2; do
  r=""
  for c in "C4 --spp=256 --only=1" "C4 --only=8" "C2 --only=1" "C2 --only=8"; do
    set -- $c
    n=${!#}; n=${n#--only=}
    XRT_LIB=$lib timeout -k 10 300 python3 tools/shard_sim.py $c --timing 2>/dev/null | tail -1 > $O/s.json
    r="$r $1/$n: $(python3 -c "import json; print(json.load(open('$O/s.json'))['shards']['$n']['shard_ms'][0])")"
  done
  echo "$lib $r"
done
