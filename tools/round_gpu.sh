#!/bin/bash
# tools/round_gpu.sh TAG [CONFIGS...] — the full GPU test suite, then tools/evidence_all.sh for
# CONFIGS (skipped when none are given).  Stops at the first failing step.
set -euo pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
if [ $# -gt 0 ]; then tools/evidence_all.sh "$TAG" "$@"; fi
