#!/bin/bash
# tools/pmc_quick.sh TAG CONFIG [LIB] — one SQ instruction-mix pass (VALU/SALU/LDS/branch/VMEM) of one
# bench frame of CONFIG, per kernel, optionally with an experiment build (variants/libxrt_hip_LIB.so)
set -uo pipefail
TAG=$1; CFG=$2; LIB=${3:-default}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG; mkdir -p "$O"; export TMPDIR=/tmp
if [ "$LIB" != default ]; then export XRT_LIB=libxrt_hip_$LIB.so; fi
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU \
  -d "$O/q_$LIB" -o q --output-format csv -- python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 0 --no-cpu --no-timing > "$O/q_$LIB.log" 2>&1 || exit $?
python3 - "$O/q_$LIB" "$LIB" <<'PY'
import collections, csv, glob, re, sys
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        if m: acc[m.group(1)][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in acc.items():
    if c.get("SQ_INSTS_VALU", 0) < 1e8: continue
    print(sys.argv[2], k, " ".join(f"{n[3:]}={v:.4g}" for n, v in sorted(c.items())))
PY
rm -rf "$O/q_$LIB"
