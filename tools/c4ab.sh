#!/bin/bash
# tools/c4ab.sh TAG — C4 parity subset, deep-queue counters of the experiment build with and
# without the bounding-ball cull (XRT_NO_BALL), and the default library's C4 bench line
set -euo pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "c4 or mesh or query or triangle_light" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for arm in ball noball; do
  if [ $arm = noball ]; then export XRT_NO_BALL=1; fi
  XRT_LIB=libxrt_hip_exp.so timeout -k 10 300 python3 bench.py --config C4 --spp 64 --steps 1 --warmup 0 --no-cpu \
    > $O/b_$arm.json 2> $O/b_$arm.err
  echo "$arm $(grep 'deep rays' $O/b_$arm.err | tail -1)"
  python3 -c "import json; d=json.load(open('$O/b_$arm.json')); print('$arm', d['value'], d['roofline']['kernel_ms_per_step'])"
done
unset XRT_NO_BALL
timeout -k 10 300 python3 bench.py --config C4 --steps 1 --warmup 1 --no-cpu > $O/b_full.json
python3 -c "import json; d=json.load(open('$O/b_full.json')); print('C4 full', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])"
