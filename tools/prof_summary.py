"""tools/prof_summary.py DIR [kernel-substring] [--traffic CONFIG OUT.json] [--pmc CONFIG OUT.json]
[--csv OUT.csv] — summarise a tools/profile.sh run: per-kernel time from the kernel trace,
summed PMC counters of the chosen kernel with derived ratios, and
  --traffic: the per-launch HBM bytes of that kernel for bench.py's roofline.traffic,
             corrected as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE (KiB) doubled on
             gfx950, WRITE_SIZE (KiB) as is, each from its own pass;
  --pmc:     per-launch SQ counters for bench.py's measured roofline (VALU issue);
  --csv:     every counter of the kernel per dispatch (the file the roofline is recomputed from)."""
import collections
import csv
import glob
import json
import os
import re
import sys


def main():
    args = sys.argv[1:]
    traffic = pmc_out = csv_out = None
    if "--traffic" in args:
        i = args.index("--traffic")
        traffic = (args[i + 1], args[i + 2])
        del args[i:i + 3]
    if "--pmc" in args:
        i = args.index("--pmc")
        pmc_out = (args[i + 1], args[i + 2])
        del args[i:i + 3]
    if "--csv" in args:
        i = args.index("--csv")
        csv_out = args[i + 1]
        del args[i:i + 2]
    d = args[0]
    # a kernel family: a name or a regex of names (e.g. "k_step_merged|k_step_spec": the merged
    # schedule's step launches, which xrt_stats times as one family), keyed by its first name
    pat = args[1] if len(args) > 1 else "k_step"
    fam = re.compile(pat)
    st = glob.glob(os.path.join(d, "kt", "*kernel_stats.csv"))
    # the kernel family's average launch: every dispatch of every instantiation whose name
    # matches (e.g. k_step_merged's 64-, 32- and 16-slot layouts), total time / total calls
    avg_ns = None
    fam_ns, fam_calls = 0.0, 0
    if st:
        for r in csv.DictReader(open(st[0])):
            print(f'{float(r["TotalDurationNs"]) / 1e6:9.3f} ms {int(r["Calls"]):6d} calls '
                  f'avg {float(r["AverageNs"]) / 1e3:9.2f} us  {r["Name"][:80]}')
            if fam.search(r["Name"]):
                fam_ns += float(r["TotalDurationNs"])
                fam_calls += int(r["Calls"])
        if fam_calls:
            avg_ns = fam_ns / fam_calls
    acc = collections.defaultdict(float)
    n = collections.Counter()
    kname = None
    rows = []
    for f in sorted(glob.glob(os.path.join(d, "*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if fam.search(r["Kernel_Name"]):
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
                n[r["Counter_Name"]] += 1
                rows.append((os.path.basename(os.path.dirname(f)), r.get("Dispatch_Id", ""), r["Counter_Name"],
                             r["Counter_Value"]))
                if kname is None:
                    m = re.search(r"(k_\w+)", pat if "|" in pat else r["Kernel_Name"])
                    kname = m.group(1) if m else pat
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
    fetch = 2 * a["FETCH_SIZE"] * 1024 if "FETCH_SIZE" in a else None
    write = a["WRITE_SIZE"] * 1024 if "WRITE_SIZE" in a else None
    if fetch is not None:
        print("FETCH_SIZE x2 (gfx950 correction) = %.3f GB" % (fetch / 1e9))
    if write is not None:
        print("WRITE_SIZE = %.3f GB" % (write / 1e9))
    if traffic and fetch is not None and write is not None:
        launches = n["FETCH_SIZE"]
        out = {"config": traffic[0], "kernel": kname, "launches": launches,
               "fetch_bytes_per_launch": fetch / launches, "write_bytes_per_launch": write / launches,
               "hbm_bytes_per_launch": (fetch + write) / launches,
               "avg_launch_us_rocprof": avg_ns / 1e3 if avg_ns else None, "rocprof_calls": fam_calls,
               "rocprof_total_ms": fam_ns / 1e6, "source": os.path.basename(d.rstrip("/")),
               "note": "FETCH_SIZE x2 + WRITE_SIZE per MI355X_MICROARCH.md HBM section; separate --pmc passes"}
        json.dump(out, open(traffic[1], "w"), indent=1)
        print("wrote", traffic[1], out)
    if pmc_out and a.get("SQ_INSTS_VALU"):
        launches = n["SQ_INSTS_VALU"]
        out = {"config": pmc_out[0], "kernel": kname, "launches": launches,
               "SQ_INSTS_VALU_per_launch": a["SQ_INSTS_VALU"] / launches,
               "avg_launch_us_rocprof": avg_ns / 1e3 if avg_ns else None, "rocprof_calls": fam_calls,
               "rocprof_total_ms": fam_ns / 1e6,
               "source": os.path.basename(d.rstrip("/"))}
        for k in ("SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_BRANCH",
                  "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY"):
            if k in a:
                out[k + "_per_launch"] = a[k] / n[k]
        if a.get("SQ_ACTIVE_INST_VALU") and a.get("SQ_THREAD_CYCLES_VALU"):
            out["lane_utilisation"] = round(a["SQ_THREAD_CYCLES_VALU"] / (64 * a["SQ_ACTIVE_INST_VALU"]), 4)
        if a.get("SQ_WAVE_CYCLES"):
            if "SQ_ACTIVE_INST_VALU" in a:
                out["valu_active_per_wave_cycle"] = round(a["SQ_ACTIVE_INST_VALU"] / a["SQ_WAVE_CYCLES"], 4)
            if "SQ_WAIT_ANY" in a:
                out["wait_per_wave_cycle"] = round(a["SQ_WAIT_ANY"] / a["SQ_WAVE_CYCLES"], 4)
        json.dump(out, open(pmc_out[1], "w"), indent=1)
        print("wrote", pmc_out[1], out)
    if csv_out and rows:
        with open(csv_out, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["pass", "dispatch_id", "counter", "value"])
            w.writerows(rows)
        print("wrote", csv_out, len(rows), "rows")


if __name__ == "__main__":
    main()
