set -u
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
grep -E "FAILED|Error" $O/gpu_tests.log | head -5
bash tools/ab.sh r05d -b "C3" -s "C3:8" -r 2 default perlane || exit $?
tools/pmc.sh r05d_pix C3 > /dev/null 2>&1; echo "pmc rc=$?"
grep "k_pixel" gpurun_out/r05d_pix/summary.txt | cut -c1-1500
rm -rf gpurun_out/r05d_pix/{kt,sq1,sq2,tcc,fetch,write}
