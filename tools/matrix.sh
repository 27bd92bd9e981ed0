set -euo pipefail
mkdir -p gpurun_out/matrix
timeout -k 10 200 python3 -u tools/shard_sim.py C2 --timing > gpurun_out/matrix/shard_c2.log 2>&1
echo shard done
for c in C3 C5; do timeout -k 10 300 python3 -u bench.py --config $c --steps 1 --warmup 1 --no-cpu > gpurun_out/matrix/bench_$c.json 2> gpurun_out/matrix/bench_$c.err; echo $c done; done
timeout -k 10 300 python3 -u bench.py --config C4 --steps 1 --warmup 0 --no-cpu > gpurun_out/matrix/bench_C4.json 2> gpurun_out/matrix/bench_C4.err
echo C4 done
