"""tools/sim/spec_sim.py [CONFIG] [STRIDE] — per-pixel chain length (visits) of the merged
schedule today vs. with speculative sample starts, from the CPU restatement's paths."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from xraytracer_amd import abi, scenes  # noqa: E402
import pyoracle  # noqa: E402

so = os.path.join(HERE, "libspec_sim.so")
subprocess.check_call(["gcc", "-O2", "-std=gnu11", "-fPIC", "-ffp-contract=off", "-fopenmp", "-w", "-shared", "-o", so,
                       os.path.join(HERE, "spec_sim.c"), "-lm"])
lib = C.CDLL(so)
cfg_name = sys.argv[1] if len(sys.argv) > 1 else "C2"
stride = int(sys.argv[2]) if len(sys.argv) > 2 else 4
cfg = scenes.CONFIGS[cfg_name]
W, H, SPP = cfg["width"], cfg["height"], cfg["spp"]
s = scenes.build(cfg_name)
pix = [(i, j) for i in range(0, H, stride) for j in range(0, W, stride)]
pi = np.array([q[0] for q in pix], np.uint32)
pj = np.array([q[1] for q in pix], np.uint32)
vis = np.zeros((len(pix), 3), np.uint32)
p = pyoracle.params(s, W, H, SPP)
u32p = C.POINTER(C.c_uint32)
lib.sim_visits(C.byref(s.desc), C.byref(pyoracle.camera(s.camera)), C.byref(p), pi.ctypes.data_as(u32p),
               pj.ctypes.data_as(u32p), len(pix), vis.ctypes.data_as(u32p))
for k, name in ((0, "today"), (1, "speculative"), (2, "enumerated")):
    v = vis[:, k]
    print(f"{name:12s} mean {v.mean():8.1f}  p99 {np.percentile(v, 99):8.1f}  max {v.max():6d}")
