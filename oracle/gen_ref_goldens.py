"""Regenerate tests/golden/ref_kats.json from the reference's own code.

TEST INFRASTRUCTURE ONLY.  Runs in the build container (where /root/reference exists):
builds oracle/_ref/ref_kats with `make -C oracle ref` (reference geometry.cpp +
sampler.cpp + headers compiled in place, see oracle/ref_kats.cpp) and stores its JSON
output.  The fixture is data (inputs and expected outputs as float bit patterns); no
reference source text is stored.

    python oracle/gen_ref_goldens.py
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "tests", "golden", "ref_kats.json")


def main():
    if not os.path.isdir("/root/reference/Src"):
        sys.exit("reference sources not present; the committed fixture stays as is")
    subprocess.check_call(["make", "-s", "-C", HERE, "ref"])
    raw = subprocess.check_output([os.path.join(HERE, "_ref", "ref_kats")])
    data = json.loads(raw)
    data["_provenance"] = ("oracle/_ref/ref_kats built by `make -C oracle ref` from "
                           "/root/reference/Src/{geometry,sampler}.cpp + headers (g++ 11.4, "
                           "-O2 -ffp-contract=off); floats stored as uint32 bit patterns")
    with open(OUT, "w") as f:
        json.dump(data, f, separators=(",", ":"))
    print("wrote", os.path.relpath(OUT), sum(len(v) for v in data.values() if isinstance(v, list)), "words")


if __name__ == "__main__":
    main()
