"""tools/spill_sites.py SRC.hip PATTERN... — where a kernel's scratch (spill) instructions sit.

Compiles SRC (gfx950, the library's flags) to assembly and, for every kernel whose mangled name
contains one of the PATTERNs, counts scratch_load / scratch_store instructions by the loop depth
the compiler annotates their basic block with (0 = outside every loop).  A spill in the
outermost loop runs once per slot batch; one at the visit loop's depth runs once per visit.
"""
import collections
import os
import re
import subprocess
import sys

src, pats = sys.argv[1], sys.argv[2:]
here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "xraytracer_amd", "csrc")
out = "/tmp/spill_sites.s"
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-I../../include",
                "-I.", "--offload-arch=gfx950", "--cuda-device-only", "-S", src, "-o", out], cwd=here, check=True,
               stderr=subprocess.DEVNULL)
asm = open(out).read()
for name in re.findall(r"^(_Z\S+):", asm, re.M):
    if not any(p in name for p in pats):
        continue
    body = asm[asm.index(name + ":"):]
    body = body[:body.index(".Lfunc_end")]
    depth, cnt, total = 0, collections.Counter(), collections.Counter()
    for line in body.splitlines():
        m = re.match(r"^\.LBB\d+_\d+:", line)
        if m:
            d = re.search(r"Depth=(\d+)", line)
            depth = int(d.group(1)) if d else 0
        t = line.strip()
        if t.startswith("scratch_"):
            cnt[depth] += 1
        if t and not t.startswith((".", ";")) and not t.endswith(":"):
            total[depth] += 1
    print(f"{name[:90]}\n  scratch instructions by loop depth: {dict(sorted(cnt.items()))}"
          f"  (all instructions by depth: {dict(sorted(total.items()))})")
