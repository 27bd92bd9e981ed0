#!/bin/bash
# tools/evidence_all.sh TAG [CONFIGS...] — tools/evidence.sh for each config (default C3 C4 C5
# C2): rocprof kernel trace + PMC passes + per-config profiles/{pmc,traffic}_CONFIG.json + the
# default bench line with its CPU baseline, into gpurun_out/TAG_CONFIG/.
set -euo pipefail
TAG=$1; shift
CFGS=${*:-C3 C4 C5 C2}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for c in $CFGS; do
  timeout -k 10 900 "$R/tools/evidence.sh" "${TAG}_$c" "$c" > "$R/gpurun_out/${TAG}_$c.log" 2>&1
  echo "$c: $(tail -1 "$R/gpurun_out/${TAG}_$c.log" | cut -c1-160)"
done
