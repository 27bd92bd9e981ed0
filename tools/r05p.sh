set -u
bash tools/ab.sh r05p -b "C3" -s "C3:8" -r 3 default untyped || exit $?
