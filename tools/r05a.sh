set -u
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests/test_gpu_pixel.py -x -v --timeout 120 --timeout-method thread > $O/pixel.log 2>&1
rc=$?; echo "pixel tests rc=$rc"; tail -3 $O/pixel.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python bench.py --config C3 --steps 3 --warmup 1 --no-cpu > $O/c3_pixel.json 2> $O/c3_pixel.err || exit $?
cat $O/c3_pixel.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['schedule'], d['roofline']['kernel_ms_per_step'])"
timeout -k 10 240 python bench.py --config C3 --steps 3 --warmup 1 --no-cpu --schedule step > $O/c3_step.json 2> $O/c3_step.err || exit $?
cat $O/c3_step.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['schedule'], d['roofline']['kernel_ms_per_step'])"
timeout -k 10 300 python tools/shard_sim.py C3 --timing > $O/c3_shards.log 2>&1 || exit $?
grep -v "^{" $O/c3_shards.log
