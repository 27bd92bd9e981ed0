#!/bin/bash
# tools/spw_sweep.sh TAG CONFIG SPP "N..." "SPW..." — shard 0 of N row shards of CONFIG at SPP under
# each forced slots-per-wave layout of the merged schedules (0 = the library's choice)
set -euo pipefail
TAG=$1; CFG=$2; SPP=$3; NS=$4; SPWS=$5
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG; mkdir -p "$O"
for n in $NS; do
  for w in $SPWS; do
    timeout -k 10 300 python3 "$R/tools/shard_sim.py" "$CFG" --spp="$SPP" --only="$n" --spw="$w" > "$O/${CFG}_n${n}_w${w}.log"
    echo "$CFG N=$n spw=$w: $(grep '^{' "$O/${CFG}_n${n}_w${w}.log" | python3 -c "import json,sys; d=json.load(sys.stdin)['shards']; print([v['shard_ms'] for v in d.values()])")"
  done
done
