"""tools/prof_summary.py DIR [kernel-substring] — summarise a tools/profile.sh run: per-kernel
time from the kernel trace, and summed PMC counters of the chosen kernel with derived
ratios (lane utilisation, wait fractions, bytes)."""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "k_step"
    st = glob.glob(os.path.join(d, "kt", "*kernel_stats.csv"))
    if st:
        for r in csv.DictReader(open(st[0])):
            print(f'{float(r["TotalDurationNs"]) / 1e6:9.3f} ms {int(r["Calls"]):6d} calls  {r["Name"][:90]}')
    acc = collections.defaultdict(float)
    n = collections.Counter()
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
                n[r["Counter_Name"]] += 1
    for k in sorted(acc):
        print(f"{k:28s} {acc[k]:.4g}  ({n[k]} dispatches)")
    a = acc
    if a.get("SQ_ACTIVE_INST_VALU"):
        print("lane utilisation  THREAD_CYCLES_VALU / (64 * ACTIVE_INST_VALU) = %.3f"
              % (a["SQ_THREAD_CYCLES_VALU"] / (64 * a["SQ_ACTIVE_INST_VALU"])))
    if a.get("SQ_WAVE_CYCLES"):
        w = a["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
            if k in a:
                print(f"{k:28s} / WAVE_CYCLES = {a[k] / w:.3f}")
    if a.get("FETCH_SIZE") is not None and "FETCH_SIZE" in a:
        print("FETCH_SIZE x2 (gfx950 correction) = %.3f GB" % (2 * a["FETCH_SIZE"] * 1024 / 1e9))
    if "WRITE_SIZE" in a:
        print("WRITE_SIZE = %.3f GB" % (a["WRITE_SIZE"] * 1024 / 1e9))


if __name__ == "__main__":
    main()
