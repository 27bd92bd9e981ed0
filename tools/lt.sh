#!/bin/bash
# tools/lt.sh — per-launch times and live counts of C2 at 1 and 8 row shards (needs the
# experiment build: make -C xraytracer_amd/csrc variant TAG=exp; XRT_TRACE_LAUNCHES)
set -euo pipefail
mkdir -p gpurun_out/lt
export XRT_LIB=libxrt_hip_exp.so
XRT_TRACE_LAUNCHES=1 timeout -k 10 120 python3 tools/shard_sim.py C2 --only=8 --timing > gpurun_out/lt/trace8.log 2>&1
XRT_TRACE_LAUNCHES=1 timeout -k 10 120 python3 tools/shard_sim.py C2 --only=1 --timing > gpurun_out/lt/trace1.log 2>&1
