set -u
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pixel.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "pixel or sphere or c3 or kstep" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $O/tests.log | head -5; exit $rc; fi
bash tools/ab.sh r05e -b "C3" -s "C3:8" -r 2 default perlane || exit $?
tools/pmc.sh r05e_pix C3 > /dev/null 2>&1; echo "pmc rc=$?"
grep "k_pixel" gpurun_out/r05e_pix/summary.txt | cut -c1-1500
rm -rf gpurun_out/r05e_pix/{kt,sq1,sq2,tcc,fetch,write}
