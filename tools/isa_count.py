"""tools/isa_count.py FILE.s [substr...] — per-kernel instruction mix of a device .s file."""
import re
import sys
from collections import Counter

txt = open(sys.argv[1]).read().split("\n")
subs = sys.argv[2:] or ["k_step_merged"]
name, body = None, []
out = []
for line in txt:
    m = re.match(r"^(_Z\w+):", line)
    if m:
        name, body = m.group(1), []
        continue
    if name and line.startswith(".Lfunc_end"):
        out.append((name, body))
        name = None
        continue
    if name and line.startswith("\t") and not line.strip().startswith((".", ";")):
        body.append(line.strip().split()[0])
for n, b in out:
    if not all(s in n for s in subs):
        continue
    c = Counter(b)
    v = sum(k for i, k in c.items() if i.startswith("v_"))
    s = sum(k for i, k in c.items() if i.startswith("s_"))
    ds = sum(k for i, k in c.items() if i.startswith("ds_"))
    g = sum(k for i, k in c.items() if i.startswith(("global_", "buffer_", "flat_")))
    print(f"{n[:70]:70s} v {v:5d} s {s:5d} ds {ds:4d} mem {g:4d} div_scale {c['v_div_scale_f32']:3d} "
          f"rcp {c['v_rcp_f32']:3d} sqrt {c['v_sqrt_f32']:3d} f64 {sum(k for i, k in c.items() if i.endswith('_f64')):4d}")
