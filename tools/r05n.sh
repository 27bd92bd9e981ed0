set -u
bash tools/ab.sh r05n -b "C3" -r 1 default noshl xnoshade xnocam xnone || exit $?
for l in xnoshade xnocam xnone; do tools/pmc_quick.sh r05n C3 $l || exit $?; done
