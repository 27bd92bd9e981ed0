set -euo pipefail
mkdir -p gpurun_out/lt
XRT_TRACE_LAUNCHES=1 timeout -k 10 120 python3 tools/shard_sim.py C2 --only=8 --timing > gpurun_out/lt/trace8.log 2>&1
XRT_STEP_VISITS=32 timeout -k 10 120 python3 tools/shard_sim.py C2 --only=8 --timing > gpurun_out/lt/v32.log 2>&1
XRT_TRACE_LAUNCHES=1 timeout -k 10 120 python3 tools/shard_sim.py C2 --only=1 --timing > gpurun_out/lt/trace1.log 2>&1
