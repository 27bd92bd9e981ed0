"""tools/phase_split.py DIR — per-phase cycle split of k_step_merged from tools/phase.sh logs.

Columns of the "[xrt] phase cycles" line (XRT_PHASE_CLOCK build, s_memtime cycles summed over
waves, lane 0): stats[8..13] = loop head (ballot), merged trace, NEE resolve + RNG take,
finish / next-sample start (camera ray), RNG prefetch, end-of-launch drain; stats[24..27]
(printed under the older "coop" label) = the shading sub-phases of the merged kernel: hit
fetch, Russian roulette + emission, light sampling (NEE), Lambert BSDF sampling.
"""
import glob
import os
import re
import sys

NAMES = ["loop head", "trace", "resolve+take", "finish/start", "prefetch", "drain",
         "hit fetch", "RR+Le", "NEE light sample", "BSDF sample"]
d = sys.argv[1]
for err in sorted(glob.glob(os.path.join(d, "s*.err")), key=lambda p: int(re.findall(r"s(\d+)", p)[-1])):
    n = re.findall(r"s(\d+)", err)[-1]
    lines = [l for l in open(err) if "phase cycles" in l]
    if not lines:
        continue
    nums = [int(x) for x in re.findall(r"\d+", lines[-1].split("sum over waves):")[1])]
    ph = nums[0:6]
    m = re.search(r"coop closest cull/scan/expand/pass (\d+) (\d+) (\d+) (\d+)", lines[-1])
    shade = [int(x) for x in m.groups()]
    cyc = ph + shade
    tot = sum(cyc)
    out = open(os.path.join(d, f"s{n}.out")).read().strip().splitlines()[-1]
    print(f"shards={n}  total {tot:.3e} wave-cycles  ({out})")
    for name, c in zip(NAMES, cyc):
        print(f"  {name:18s} {c:.3e}  {100.0 * c / tot:5.1f}%")
