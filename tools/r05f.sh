set -u
bash tools/ab.sh r05f -b "C3" -r 1 default noshade nosum notrace || exit $?
for l in default noshade nosum notrace; do tools/pmc_quick.sh r05f C3 $l || exit $?; done
