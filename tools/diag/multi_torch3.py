"""Diagnose: several live contexts (streams) before torch's own HIP runtime initialises."""
import sys
sys.path.insert(0, ".")
from xraytracer_amd import scenes
from xraytracer_amd.renderer import HipRenderer
k = int(sys.argv[1])
rs = [HipRenderer(2, device=0) for _ in range(k)]
for r in rs:
    r.render(scenes.cornell(16, 12), 16, 12)
print("contexts alive:", k, flush=True)
import torch
try:
    x = torch.zeros(4, device="cuda:0")
    print("torch ok", flush=True)
except Exception as e:
    print("torch FAILED", str(e)[:80], flush=True)
