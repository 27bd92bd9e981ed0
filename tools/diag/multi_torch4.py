"""Diagnose: torch import / HIP init order against libxrt_hip's contexts."""
import sys
sys.path.insert(0, ".")
mode = sys.argv[1]
if mode in ("import_first", "init_first"):
    import torch
    if mode == "init_first":
        torch.zeros(1, device="cuda:0")
from xraytracer_amd import scenes
from xraytracer_amd.renderer import HipRenderer
rs = [HipRenderer(2, device=0), HipRenderer(2, devices=[0, 0])]
for r in rs:
    r.render(scenes.cornell(16, 12), 16, 12)
import torch
try:
    x = torch.zeros(4, device="cuda:0")
    rs[1].render_device(scenes.cornell(16, 12), 16, 12, torch.zeros(12, 16, 3, device="cuda:0").data_ptr())
    print(mode, "torch ok", flush=True)
except Exception as e:
    print(mode, "torch FAILED", str(e)[:80], flush=True)
