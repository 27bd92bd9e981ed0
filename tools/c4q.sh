#!/bin/bash
# tools/c4q.sh TAG — C4 parity subset (default library), then the deep walk one lane per ray
# vs four (experiment build, XRT_DEEP_QUAD=0/1): C4 at 256 spp on one GPU and shard 0 of 8
set -euo pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "c4 or mesh or query or triangle_light" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for qd in 0 1; do
  XRT_DEEP_QUAD=$qd XRT_LIB=libxrt_hip_exp.so timeout -k 10 300 python3 bench.py --config C4 --spp 256 --steps 1 \
    --warmup 0 --no-cpu > $O/b$qd.json 2> $O/b$qd.err
  echo "quad=$qd $(grep 'deep rays' $O/b$qd.err | tail -1)"
  python3 -c "import json; d=json.load(open('$O/b$qd.json')); print('quad=$qd 1 GPU', d['value'], d['roofline']['kernel_ms_per_step'])"
  XRT_DEEP_QUAD=$qd XRT_LIB=libxrt_hip_exp.so timeout -k 10 300 python3 tools/shard_sim.py C4 --only=8 --timing \
    2>/dev/null | tail -1 > $O/s$qd.json
  python3 -c "import json; d=json.load(open('$O/s$qd.json'))['shards']['8']; print('quad=$qd 8 shards', d['shard_ms'], d['kernel_ms'])"
done
