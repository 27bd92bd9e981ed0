set -u
bash tools/ab.sh r05l -T "two_level or c4 or mesh or c1_cornell or merged or c2_headline" -b "C2 C4:64" -s "C2:8 C4:8:64" -r 2 default nocam trimajor || exit $?
