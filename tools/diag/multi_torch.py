"""Diagnose: does creating / rendering with a multi-device context break torch's HIP init?"""
import ctypes as C
import sys
sys.path.insert(0, ".")
from xraytracer_amd import scenes
from xraytracer_amd.renderer import HipRenderer

hip = C.CDLL("libamdhip64.so")
def count(tag):
    n = C.c_int(-1)
    rc = hip.hipGetDeviceCount(C.byref(n))
    print(tag, "hipGetDeviceCount rc", rc, "n", n.value, flush=True)

mode = sys.argv[1]
count("start")
if mode in ("create", "render"):
    m = HipRenderer(2, devices=[0, 0])
    count("after create_multi")
    if mode == "render":
        s = scenes.cornell(32, 24)
        m.render(s, 32, 24)
        count("after render")
if mode == "single":
    r = HipRenderer(2, device=0)
    r.render(scenes.cornell(32, 24), 32, 24)
    count("after single render")
import torch
print("torch count", torch.cuda.device_count(), flush=True)
x = torch.zeros(4, device="cuda:0")
print("torch ok", x.sum().item(), flush=True)
