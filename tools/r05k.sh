set -u
bash tools/ab.sh r05k -T "c1_cornell or merged or two_level or c2_headline" -b "C2 C4:64" -s "C2:8" -r 2 default trimajor || exit $?
for l in default trimajor; do tools/pmc_quick.sh r05k C2 $l || exit $?; done
