#!/bin/bash
# tools/round_end.sh TAG STAGE — a round's GPU evidence in stages that each fit one gpurun call:
#   tests   the full GPU suite + smoke()                   -> gpurun_out/TAG/{gpu_tests,smoke}.log
#   ev CFG… tools/evidence.sh per config (rocprof kernel stats, PMC passes, bench line + CPU baseline)
#   shards CFG…  tools/shard_sim.py per config (shard 0 and N-1 of N = 1, 2, 4, 8) -> gpurun_out/TAG/shard_CFG.json
# Every GPU step has its own time limit; the script stops at the first failure.
set -euo pipefail
TAG=$1; STAGE=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG; mkdir -p "$O"
case $STAGE in
  tests)
    timeout -k 10 700 python3 -u -m pytest "$R/tests" -m gpu -x -q --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1 \
      || { tail -30 "$O/gpu_tests.log"; exit 1; }
    tail -1 "$O/gpu_tests.log"
    (cd "$R" && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()") > "$O/smoke.log" 2>&1 \
      || { tail -20 "$O/smoke.log"; exit 1; }
    tail -2 "$O/smoke.log" ;;
  ev)
    for c in "$@"; do
      timeout -k 10 900 "$R/tools/evidence.sh" "${TAG}_$c" "$c" > "$O/ev_$c.log" 2>&1 || { tail -20 "$O/ev_$c.log"; exit 1; }
      echo "$c: $(tail -1 "$O/ev_$c.log" | cut -c1-200)"
    done ;;
  shards)
    for c in "$@"; do
      timeout -k 10 600 python3 "$R/tools/shard_sim.py" "$c" > "$O/shard_$c.log" 2>&1 || { tail -20 "$O/shard_$c.log"; exit 1; }
      tail -1 "$O/shard_$c.log" > "$O/shard_$c.json"
      cat "$O/shard_$c.json"
    done ;;
  *) echo "unknown stage $STAGE"; exit 2 ;;
esac
