"""Diagnose: replay test_multi_matches_single_and_oracle, then init torch."""
import ctypes as C
import sys
sys.path.insert(0, "."); sys.path.insert(0, "oracle")
import numpy as np
import pyoracle
from xraytracer_amd import abi, scenes
from xraytracer_amd.renderer import HipRenderer

hip = C.CDLL("libamdhip64.so")
def count(tag):
    n = C.c_int(-1)
    rc = hip.hipGetDeviceCount(C.byref(n))
    print(tag, "hipGetDeviceCount rc", rc, "n", n.value, flush=True)

single = HipRenderer(4, device=0)
for n in (2, 3):
    s = scenes.cornell(96, 71)
    m = HipRenderer(4, devices=[0] * n)
    count(f"n={n} created")
    img = m.render(s, 96, 71, timing=True)
    count(f"n={n} rendered")
    part = m.render(s, 96, 71, shard_index=1, shard_count=2)
    count(f"n={n} shard rendered")
    m.close()
    count(f"n={n} closed")
import torch
print("torch count", torch.cuda.device_count(), flush=True)
x = torch.zeros(4, device="cuda:0")
print("torch ok", x.sum().item(), flush=True)
