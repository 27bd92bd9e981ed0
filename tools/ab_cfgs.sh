#!/bin/bash
# tools/ab_cfgs.sh TAG LIB... — frame times (tools/shard_sim.py) of the default library and
# each plain experiment build LIB on: C4 256 spp one GPU, C4 shard 0 of 8, C2 one GPU,
# C2 shard 0 of 8, C3 one GPU, C5 one GPU (set AB_CASES to override: CONFIG:ARG,ARG:N ...)
set -euo pipefail
O=gpurun_out/$1; shift; mkdir -p $O
CASES=${AB_CASES:-"C4:--spp=256:1 C4::8 C2::1 C2::8 C3::1 C5::1"}
for lib in libxrt_hip.so "$@"; do
  r=""
  for c in $CASES; do
    IFS=: read -r cfg extra n <<< "$c"
    extra=${extra//,/ }   # several extra arguments are comma-separated within a case
    XRT_LIB=$lib timeout -k 10 300 python3 tools/shard_sim.py $cfg $extra --only=$n --timing 2>/dev/null | tail -1 > $O/s.json
    r="$r $cfg/$n: $(python3 -c "import json; print(json.load(open('$O/s.json'))['shards']['$n']['shard_ms'][0])")"
  done
  echo "$lib $r"
done
