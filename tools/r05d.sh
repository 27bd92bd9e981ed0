set -u
bash tools/ab.sh r05d -b "C3" -s "C3:8" -r 2 default perlane || exit $?
tools/pmc.sh r05d_pix C3 > /dev/null 2>&1; echo "pmc rc=$?"
grep "k_pixel" gpurun_out/r05d_pix/summary.txt | cut -c1-1500
rm -rf gpurun_out/r05d_pix/{kt,sq1,sq2,tcc,fetch,write}
