#!/bin/bash
# tools/pmc_shard.sh TAG CONFIG N [shard_sim args] — one SQ instruction-mix pass over shard 0 of N row shards of
# CONFIG (tools/shard_sim.py --only=N: a warm-up render and the timed one), per kernel
# instantiation: launches, VALU / SALU / LDS / VMEM / branch instructions per launch, wait and
# VALU-active shares of the wave cycles
set -uo pipefail
TAG=$1; CFG=$2; N=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG; mkdir -p "$O"; export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU \
  -d "$O/ps" -o q --output-format csv -- python3 "$R/tools/shard_sim.py" "$CFG" --only="$N" --reps=1 --warm-shard "$@" > "$O/ps_${CFG}_$N.log" 2>&1 || exit $?
python3 - "$O/ps" > "$O/pmc_shard_${CFG}_$N.txt" <<'PY'
import collections, csv, glob, sys
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    seen = set()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:110]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if (r["Dispatch_Id"], k) not in seen:
            seen.add((r["Dispatch_Id"], k)); n[k] += 1
for k, c in sorted(acc.items(), key=lambda x: -x[1].get("SQ_INSTS_VALU", 0)):
    if c.get("SQ_INSTS_VALU", 0) < 1e6: continue
    L = n[k]; wc = max(c.get("SQ_WAVE_CYCLES", 1), 1)
    print(f"{k}\n   launches {L}  per launch: VALU {c['SQ_INSTS_VALU']/L:.4g} SALU {c['SQ_INSTS_SALU']/L:.4g} "
          f"LDS {c['SQ_INSTS_LDS']/L:.4g} VMEM_RD {c['SQ_INSTS_VMEM_RD']/L:.4g} BRANCH {c['SQ_INSTS_BRANCH']/L:.4g}  "
          f"wait {c['SQ_WAIT_ANY']/wc:.3f} valu-active {c['SQ_ACTIVE_INST_VALU']/wc:.3f}")
PY
rm -rf "$O/ps"
cat "$O/pmc_shard_${CFG}_$N.txt"

