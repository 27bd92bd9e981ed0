"""tools/shard_sim.py [CONFIG] — predict strong scaling on one GPU.

Renders shard 0 (and the last shard) of N = 1, 2, 4, 8 row shards of CONFIG on cuda:0 and
prints the per-shard frame time and the implied whole-node Msamples/s (W*H*spp / slowest shard
time).  The multi-GPU bench runs exactly these shards, one per GPU, plus the frame assembly on
rank 0; this isolates the per-GPU part and estimates the assembly.

One harness for every point: a full-frame render warms the context first (its
buffers are sized by the largest shard, the whole frame), then every point is the MEDIAN of
--reps renders (default 3), host clock around render_device + synchronize, as bench.py times a
step.  ratio_vs_1 divides this harness's own N = 1 median.

Assembly estimate (the RCCL gather bench.py runs for N > 1; it cannot run on one GPU): rank 0's
device-side share measured here — packing its own rows and writing the N - 1 received shards
into place (torch strided copies of the real frame) — plus a modelled transfer: the N - 1
packed shards (ceil(H/N) x W x 12 B each) arrive over N - 1 separate xGMI links in parallel at
an assumed LINK_GBS effective rate, plus COLLECTIVE_US of fixed collective latency.
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LINK_GBS = 100.0       # assumed effective GB/s of one xGMI link (peak ~153 GB/s per link)
COLLECTIVE_US = 50.0   # assumed fixed latency of one RCCL gather


def assembly_device_ms(fb, n, reps):
    """Rank 0's strided copies of a gather of n shards: pack own rows, unpack n - 1 shards."""
    import torch
    H = fb.shape[0]
    rmax = (H + n - 1) // n
    bufs = [fb.new_zeros((rmax,) + tuple(fb.shape[1:])) for _ in range(n)]
    times = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mine = fb[0::n]
        bufs[0][: mine.shape[0]] = mine
        for r in range(1, n):
            k = len(range(r, H, n))
            fb[r::n] = bufs[r][:k]
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    return statistics.median(times) * 1e3


def main():
    import torch
    from xraytracer_amd import abi, distributed, scenes
    from xraytracer_amd.renderer import HipRenderer

    cfg_name = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else "C2"
    timing = "--timing" in sys.argv
    only = [int(a.split("=")[1]) for a in sys.argv if a.startswith("--only=")]
    spw = ([int(a.split("=")[1]) for a in sys.argv if a.startswith("--spw=")] or [0])[0]
    reps = ([int(a.split("=")[1]) for a in sys.argv if a.startswith("--reps=")] or [3])[0]
    group = "--no-group" not in sys.argv
    deep = ([a.split("=")[1] for a in sys.argv if a.startswith("--deep=")] or ["auto"])[0]
    sched = ([a.split("=")[1] for a in sys.argv if a.startswith("--schedule=")] or ["auto"])[0]
    cfg = scenes.CONFIGS[cfg_name]
    W, H, SPP = cfg["width"], cfg["height"], cfg["spp"]
    SPP = ([int(a.split("=")[1]) for a in sys.argv if a.startswith("--spp=")] or [SPP])[0]
    scene = scenes.build(cfg_name)
    if "--sparse" in sys.argv:   # media: upload the grid as 8^3 leaf bricks (same image)
        scene.medium.sparse = True
    r = HipRenderer(SPP, device=0)
    r.upload(scene)
    fb = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda:0")
    kw = dict(slots_per_wave=spw, group=group, deep=deep, schedule=sched, spec="--no-spec" not in sys.argv)
    # warm: full-frame buffers (--warm-shard: the first measured shard instead, so a counter
    # pass over the run sees that shard's launches only)
    wn = (only[0] if only else 1) if "--warm-shard" in sys.argv else 1
    r.render_device(scene, W, H, fb.data_ptr(), shard_index=0, shard_count=wn, **kw)
    torch.cuda.synchronize()
    res = {}
    for n in (only or (1, 2, 4, 8)):
        shards = {}
        st = None
        for s in (sorted({0, n - 1}) if not only else [0]):
            times = []
            for _ in range(reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                st = r.render_device(scene, W, H, fb.data_ptr(), shard_index=s, shard_count=n, timing=timing, **kw)
                torch.cuda.synchronize()
                times.append(time.perf_counter() - t0)
            shards[s] = times
        med = {s: statistics.median(t) for s, t in shards.items()}
        slow = max(med.values())
        point = {"shard_ms": [round(med[s] * 1e3, 3) for s in sorted(med)],
                 "shard_ms_all": {str(s): [round(t * 1e3, 3) for t in v] for s, v in shards.items()},
                 "kernel_ms": {abi.KERNEL_NAMES[i]: round(st.kernel_ms[i], 2) for i in range(abi.XRT_K_COUNT)
                               if st.kernel_ms[i]},
                 "msamples_s": round(W * H * SPP / slow / 1e6, 1), "iterations": int(st.iterations),
                 "schedule": abi.SCHEDULE_NAMES[st.schedule]}
        if n > 1:
            dev_ms = assembly_device_ms(fb, n, reps)
            shard_bytes = ((H + n - 1) // n) * W * 12
            link_ms = shard_bytes / (LINK_GBS * 1e9) * 1e3 + COLLECTIVE_US / 1e3
            est = dev_ms + link_ms
            point["assembly"] = {"mode": "gather", "bytes": distributed.assembly_bytes(H, W, n),
                                 "device_copies_ms": round(dev_ms, 4), "transfer_model_ms": round(link_ms, 4),
                                 "estimate_ms": round(est, 4),
                                 "model": f"{shard_bytes} B per rank over its own link at {LINK_GBS} GB/s "
                                          f"+ {COLLECTIVE_US} us collective latency (assumed, not measured)"}
            point["frame_ms_with_assembly"] = round(slow * 1e3 + est, 3)
        res[n] = point
        print(n, point, flush=True)
    base = res.get(1, {}).get("shard_ms")
    if base:
        for n, p in res.items():
            p["ratio_vs_1"] = round(max(base) / max(p["shard_ms"]), 3)
            if "frame_ms_with_assembly" in p:
                p["ratio_vs_1_with_assembly"] = round(max(base) / p["frame_ms_with_assembly"], 3)
    print(json.dumps({"config": cfg_name, "spp": SPP, "reps": reps, "harness": "median of reps, after a full-frame warm "
                      "render", "shards": res}))
    r.close()


if __name__ == "__main__":
    main()
