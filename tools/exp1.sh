set -euo pipefail
tools/costmap.sh r03cm2 libxrt_hip_cstart.so
O=gpurun_out/r03cm2
for n in 8 128 16 32; do
  timeout -k 10 200 python3 tools/shard_sim.py C2 --only=$n --timing --spw=8 2>/dev/null | tail -1 > $O/spw8_$n.json
  python3 -c "import json; d=json.load(open('$O/spw8_$n.json'))['shards']['$n']; print('spw8', $n, d['shard_ms'])"
done
