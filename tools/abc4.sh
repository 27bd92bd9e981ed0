#!/bin/bash
# tools/abc4.sh TAG LIB — C4 parity subset (default library), then C4 one GPU (256 spp) and
# shard 0 of 8 (full spp), default library vs LIB (a plain `make variant EXP=` build)
set -euo pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "c4 or mesh or query or triangle_light" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for lib in libxrt_hip.so $2; do
  XRT_LIB=$lib timeout -k 10 300 python3 bench.py --config C4 --spp 256 --steps 1 --warmup 1 --no-cpu > $O/b_$lib.json
  XRT_LIB=$lib timeout -k 10 300 python3 tools/shard_sim.py C4 --only=8 --timing 2>/dev/null | tail -1 > $O/s_$lib.json
  python3 -c "
import json; b=json.load(open('$O/b_$lib.json')); s=json.load(open('$O/s_$lib.json'))['shards']['8']
print('$lib', '1 GPU', b['value'], b['roofline']['kernel_ms_per_step'], '| 8 shards', s['shard_ms'], s['kernel_ms'])"
done
