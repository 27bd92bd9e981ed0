#!/bin/bash
# tools/c3probe.sh TAG — where an 8-shard C3 frame goes: per-launch times (experiment
# build), visits-per-launch sweep, then the PMC instruction mix of shard 0 of 8
set -euo pipefail
O=gpurun_out/$1; mkdir -p $O
tools/launches.sh $1/l C3
for v in 8 16 32; do
  XRT_LIB=libxrt_hip_exp.so XRT_VISITS=$v timeout -k 10 200 python3 tools/shard_sim.py C3 --only=8 --timing 2>/dev/null | tail -1 > $O/v$v.json
  python3 -c "import json; d=json.load(open('$O/v$v.json'))['shards']['8']; print('visits $v', d['shard_ms'], d['iterations'], d['kernel_ms'])"
done
tools/pmc_shard.sh 8 $1/pmc C3
