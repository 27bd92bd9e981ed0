"""tools/phase_split.py DIR — per-phase share of k_step_spec's wave cycles from tools/phase.sh logs.

The "[xrt] spec phase cycles" line (XRT_PHASE_CLOCK build: shader-clock cycles between phase
boundaries, summed over waves, the last render of the run = the measured shard) names the phases
of a visit in order — loop head, trace (the quad's three rays), candidates (camera rays at the
three offsets + camera-list tests), end test, shading (A and B), moves (the quad's new state),
cursor + RNG reload — plus the launch prologue / epilogue.  Cycles of co-resident waves overlap,
so the shares, not the sums, compare.
"""
import glob
import os
import re
import sys

d = sys.argv[1]
for err in sorted(glob.glob(os.path.join(d, "s*.err")), key=lambda p: int(re.findall(r"s(\d+)", p)[-1])):
    n = re.findall(r"s(\d+)", err)[-1]
    lines = [l for l in open(err) if "spec phase cycles" in l]
    if not lines:
        continue
    pairs = re.findall(r"([a-z+\-]+) (\d+)", lines[-1].split("spec phase cycles")[1])
    tot = sum(int(v) for _, v in pairs)
    print(f"shards={n}  total {tot:.3e} wave-cycles")
    for name, v in pairs:
        print(f"  {name:16s} {int(v) / tot:6.1%}")
