set -u
tools/pmc.sh r05b_pix C3 > /dev/null 2>&1; echo "pmc rc=$?"
cat gpurun_out/r05b_pix/summary.txt | cut -c1-1500
rm -rf gpurun_out/r05b_pix/{kt,sq1,sq2,tcc,fetch,write}
