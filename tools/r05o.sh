set -u
O=gpurun_out/r05o; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pixel.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" $O/tests.log | head -8; exit $rc; fi
bash tools/ab.sh r05o -b "C3" -s "C3:8" -r 2 default || exit $?
tools/pmc_quick.sh r05o C3 default || exit $?
