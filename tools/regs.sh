#!/bin/bash
# tools/regs.sh [pattern] — per-kernel VGPR/SGPR/spill/occupancy of $SRC (default wavefront.hip;
# SRC=step_tri.hip for the merged kernels), gfx950; extra -D flags in $REGS_DEFS
cd "$(dirname "$0")/../xraytracer_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -I../../include -I. --offload-arch=gfx950 \
    $REGS_DEFS -c ${SRC:-wavefront.hip} -o /tmp/regs_wf.o -Rpass-analysis=kernel-resource-usage 2>&1 |
python3 -c '
import re, sys
pat = sys.argv[1] if len(sys.argv) > 1 else ""
cur = None; rows = []
for line in sys.stdin:
    m = re.search(r"remark: (?:\s*)([A-Za-z ]+[A-Za-z\]]*?)(?: \[bytes/block\])?: (\S+)", line)
    if not m: continue
    k, v = m.group(1).strip(), m.group(2)
    if k == "Function Name": cur = {"name": v}; rows.append(cur)
    elif cur is not None: cur[k] = v
for r in rows:
    if pat in r["name"]:
        print("%-60s vgpr %4s sgpr %4s sspill %3s vspill %3s occ %s lds %s" % (r["name"][:60], r.get("VGPRs"), r.get("TotalSGPRs"),
              r.get("SGPRs Spill"), r.get("VGPRs Spill"), r.get("Occupancy [waves/SIMD]"), r.get("LDS Size")))
' "$1"
