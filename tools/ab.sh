#!/bin/bash
# tools/ab.sh TAG [-t TESTSEL] [-b "CFG[:SPP] ..."] [-s "CFG:N[:SPP] ..."] [-w SCHED] [-r REPS] LIB...
# A/B runner on one GPU box: for each library LIB ("default" = xraytracer_amd/libxrt_hip.so,
# else an experiment build xraytracer_amd/variants/libxrt_hip_LIB.so from `make variant`):
#   -t  GPU parity tests selected by `pytest -k TESTSEL` (first library only: results never depend
#       on an experiment's schedule knobs, and every variant must still pass: use -T for all)
#   -b  one bench.py frame per config (optionally at SPP samples), JSON -> gpurun_out/TAG/LIB_CFG.json
#   -s  shard 0 of N row shards (tools/shard_sim.py --only=N) per config
#   -w  schedule for -s / -b (auto | wavefront)
#   -r  repetitions of the -b / -s measurements, libraries interleaved (default 1)
# Each step runs under its own time limit; the script stops at the first failure.
set -euo pipefail
TAG=$1; shift
TESTS=""; ALLTESTS=0; BENCH=""; SHARDS=""; SCHED=auto; REPS=1
while getopts "t:T:b:s:w:r:" o; do
  case $o in
    t) TESTS=$OPTARG ;; T) TESTS=$OPTARG; ALLTESTS=1 ;; b) BENCH=$OPTARG ;; s) SHARDS=$OPTARG ;;
    w) SCHED=$OPTARG ;; r) REPS=$OPTARG ;; *) exit 2 ;;
  esac
done
shift $((OPTIND - 1))
LIBS=${*:-default}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG; mkdir -p "$O"
use() { if [ "$1" = default ]; then unset XRT_LIB; else export XRT_LIB=libxrt_hip_$1.so; fi; }
first=1
for lib in $LIBS; do
  if [ -n "$TESTS" ] && { [ $first = 1 ] || [ $ALLTESTS = 1 ]; }; then
    use "$lib"
    timeout -k 10 600 python3 -u -m pytest "$R/tests" -m gpu -x -q -k "$TESTS" --timeout 200 --timeout-method thread \
      > "$O/tests_$lib.log" 2>&1 || { tail -30 "$O/tests_$lib.log"; exit 1; }
    echo "tests [$lib]: $(tail -1 "$O/tests_$lib.log")"
  fi
  first=0
done
for rep in $(seq 1 "$REPS"); do
  for lib in $LIBS; do
    use "$lib"
    for b in $BENCH; do
      cfg=${b%%:*}; spp=""; [ "$b" != "$cfg" ] && spp="--spp ${b#*:}"
      timeout -k 10 600 python3 "$R/bench.py" --config "$cfg" $spp --steps 1 --warmup 1 --no-cpu --schedule "$SCHED" \
        > "$O/${lib}_${cfg}_$rep.json"
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('$lib $b', d['value'], 'Msamples/s', d['ms_per_step'], 'ms', d['config']['schedule'])" "$O/${lib}_${cfg}_$rep.json"
    done
    for s in $SHARDS; do
      IFS=: read -r cfg n spp <<< "$s"
      timeout -k 10 600 python3 "$R/tools/shard_sim.py" "$cfg" --only="$n" ${spp:+--spp=$spp} --schedule="$SCHED" \
        > "$O/${lib}_${cfg}_s${n}_$rep.log"
      echo "$lib $s: $(grep '^{' "$O/${lib}_${cfg}_s${n}_$rep.log" | python3 -c "import json,sys; d=json.load(sys.stdin)['shards']; print({k: v['shard_ms'] for k, v in d.items()})")"
    done
  done
done
