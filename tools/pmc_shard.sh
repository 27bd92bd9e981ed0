#!/bin/bash
# tools/pmc_shard.sh N TAG [CONFIG] — PMC instruction mix of the fused kernel for shard 0 of N (C2),
# each counter group in its own rocprofv3 pass (MI355X_MICROARCH.md: no --pmc with tracing).
set -euo pipefail
N=${1:-8}; TAG=${2:-pmc}; CFG=${3:-C2}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
B=(python3 "$R/tools/shard_sim.py" "$CFG" "--only=$N")
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- "${B[@]}" > "$OUT/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d "$OUT/sq1" -o sq1 --output-format csv -- "${B[@]}" > "$OUT/sq1.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
    SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM -d "$OUT/sq2" -o sq2 --output-format csv -- "${B[@]}" > "$OUT/sq2.log" 2>&1
python3 "$R/tools/prof_summary.py" "$OUT" k_step > "$OUT/summary.txt"
cat "$OUT/summary.txt"
