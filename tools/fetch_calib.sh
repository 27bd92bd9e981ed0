#!/bin/bash
# tools/fetch_calib.sh TAG [CONFIG...] — FETCH_SIZE calibration on known byte counts
# (tools/fetch_calib.hip), then the same TCC read-request decomposition for one bench frame of
# each CONFIG: pass 1 FETCH_SIZE (on gfx950 = TCC_BUBBLE*128 + (RDREQ-BUBBLE-RDREQ_32B)*64 +
# RDREQ_32B*32, and TCC_BUBBLE reads 0), pass 2 the read requests by size (TCC_EA0_RDREQ,
# _RDREQ_64B, _RDREQ_128B) and the DRAM-bound reads in 32-B units (TCC_EA0_RDREQ_DRAM_32B).
# Sized bytes = 32*(RDREQ-64B-128B) + 64*64B + 128*128B.
# Output: gpurun_out/TAG/fetch_calib.txt
set -uo pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG; mkdir -p "$O"; export TMPDIR=/tmp
B=$R/tools/fetch_calib
P2="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_DRAM_32B_sum"
timeout -k 10 120 "$B" > "$O/calib_bytes.jsonl" || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$O/c1" -o c --output-format csv -- "$B" > /dev/null || exit $?
timeout -s KILL 90 rocprofv3 --pmc $P2 -d "$O/c2" -o c --output-format csv -- "$B" > /dev/null || exit $?
for C in "$@"; do
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$O/b1_$C" -o c --output-format csv -- python3 "$R/bench.py" \
      --config "$C" --steps 1 --warmup 0 --no-cpu --no-timing > "$O/b1_$C.log" 2>&1 || exit $?
  timeout -s KILL 200 rocprofv3 --pmc $P2 -d "$O/b2_$C" -o c --output-format csv -- python3 "$R/bench.py" \
      --config "$C" --steps 1 --warmup 0 --no-cpu --no-timing > "$O/b2_$C.log" 2>&1 || exit $?
done
python3 - "$O" "$@" > "$O/fetch_calib.txt" <<'PY'
import collections, csv, glob, json, os, re, sys
O = sys.argv[1]
def per_dispatch(d, pat):
    rows = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(O, d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if not re.search(pat, r["Kernel_Name"]): continue
            x = rows[int(r["Dispatch_Id"])]
            x["name"] = r["Kernel_Name"]
            x[r["Counter_Name"]] = x.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [rows[k] for k in sorted(rows)]
def terms(a, b):
    f = a.get("FETCH_SIZE", 0) * 1024
    rq, r64, r128 = b.get("TCC_EA0_RDREQ_sum", 0), b.get("TCC_EA0_RDREQ_64B_sum", 0), b.get("TCC_EA0_RDREQ_128B_sum", 0)
    sized = 32 * (rq - r64 - r128) + 64 * r64 + 128 * r128
    return f, rq, r64, r128, sized, 32 * b.get("TCC_EA0_RDREQ_DRAM_32B_sum", 0)
known = [json.loads(x) for x in open(os.path.join(O, "calib_bytes.jsonl"))]
pat = r"k_stream16|k_rand|k_ring32"
A, Bp = per_dispatch("c1", pat), per_dispatch("c2", pat)
print("calibration kernels (bytes per dispatch, GB): known | FETCH_SIZE | sized requests | DRAM_32B*32;"
      " requests 32/64/128 B")
for k, a, b in zip(known, A, Bp):
    f, rq, r64, r128, sized, dram = terms(a, b)
    kb = k["bytes"]
    print(f"{k['kernel']:10s} table {k.get('table', 0) / 2**20:6.0f} MiB  known {kb / 1e9:7.3f}  FETCH_SIZE {f / 1e9:7.3f}"
          f" ({f / kb:.3f}x)  sized {sized / 1e9:7.3f} ({sized / kb:.3f}x)  DRAM {dram / 1e9:7.3f} ({dram / kb:.3f}x)"
          f"  req {rq - r64 - r128:.3g}/{r64:.3g}/{r128:.3g}")
for C in sys.argv[2:]:
    A, Bp = per_dispatch("b1_" + C, r"k_"), per_dispatch("b2_" + C, r"k_")
    agg = collections.defaultdict(lambda: [0.0] * 7)
    for a, b in zip(A, Bp):
        m = re.search(r"(k_\w+)", a.get("name", ""))
        k = m.group(1) if m else "?"
        g = agg[k]; g[0] += 1
        for i, v in enumerate(terms(a, b)): g[1 + i] += v
    print(f"\n{C}: per kernel family, per launch (GB): FETCH_SIZE | x2 (guide) | sized requests | DRAM_32B*32;"
          " share of requests 32/64/128 B")
    for k, (n, f, rq, r64, r128, sized, dram) in sorted(agg.items(), key=lambda x: -x[1][1]):
        if f < 1e6: continue
        print(f"  {k:16s} {int(n):4d} launches  {f / n / 1e9:7.3f} | {2 * f / n / 1e9:7.3f} | {sized / n / 1e9:7.3f} | "
              f"{dram / n / 1e9:7.3f}   {(rq - r64 - r128) / max(rq, 1):.2f}/{r64 / max(rq, 1):.2f}/{r128 / max(rq, 1):.2f}")
PY
tar czf "$O/pmc_raw.tgz" -C "$O" c1 c2 $(cd "$O" && ls -d b1_* b2_* 2>/dev/null) && rm -rf "$O"/c1 "$O"/c2 "$O"/b1_* "$O"/b2_*
cat "$O/fetch_calib.txt"
