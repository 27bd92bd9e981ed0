#!/bin/bash
# tools/isa.sh OUT.s [DEFS] — device assembly of step_tri.hip (gfx950) for instruction counts
cd "$(dirname "$0")/../xraytracer_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -I../../include -I. --offload-arch=gfx950 \
    --cuda-device-only -S $2 step_tri.hip -o "$1"
