#!/bin/bash
# tools/profile.sh CONFIG TAG [extra bench args] — rocprofv3 evidence for one bench workload:
#   1. --kernel-trace --stats      -> per-dispatch durations + per-kernel summary
#   2. --pmc SQ timing counters    -> wave-cycle breakdown
#   3. --pmc SQ instruction mix    -> VALU / LDS instructions, LDS bank conflicts
#   4. --pmc FETCH_SIZE, 5. --pmc WRITE_SIZE (separate passes, MI355X_MICROARCH.md §HBM)
# Each pass runs bench.py once (1 step, no warmup, no CPU baseline) under its own timeout.
set -euo pipefail
CFG=${1:-C2}; TAG=${2:-prof}; shift 2 || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
B=(python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 0 --no-cpu --no-timing "$@")
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- "${B[@]}" > "$OUT/kt.log" 2>&1
echo "kernel trace done"
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS \
    -d "$OUT/sq1" -o sq1 --output-format csv -- "${B[@]}" > "$OUT/sq1.log" 2>&1
echo "sq1 done"
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
    SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM \
    -d "$OUT/sq2" -o sq2 --output-format csv -- "${B[@]}" > "$OUT/sq2.log" 2>&1
echo "sq2 done"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- "${B[@]}" > "$OUT/fetch.log" 2>&1
echo "fetch done"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- "${B[@]}" > "$OUT/write.log" 2>&1
echo "write done"
