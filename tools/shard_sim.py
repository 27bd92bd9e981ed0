"""tools/shard_sim.py [CONFIG] — predict strong scaling on one GPU.

Renders shard 0 (and the slowest of a few shards) of N = 1, 2, 4, 8 row shards of CONFIG on
cuda:0 and prints the per-shard frame time and the implied whole-node Msamples/s
(W*H*spp / slowest shard time).  The multi-GPU bench runs exactly these shards, one per
GPU, plus one RCCL reduce of the framebuffer; this isolates the per-GPU part.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from xraytracer_amd import abi, scenes
    from xraytracer_amd.renderer import HipRenderer

    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "C2"
    timing = "--timing" in sys.argv
    only = [int(a.split("=")[1]) for a in sys.argv if a.startswith("--only=")]
    spw = ([int(a.split("=")[1]) for a in sys.argv if a.startswith("--spw=")] or [0])[0]
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
    r.render_device(scene, W, H, fb.data_ptr(), shard_index=0, shard_count=8)  # warm
    res = {}
    for n in (only or (1, 2, 4, 8)):
        times = []
        for s in (sorted({0, n - 1}) if not only else [0]):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st = r.render_device(scene, W, H, fb.data_ptr(), shard_index=s, shard_count=n, timing=timing,
                                 slots_per_wave=spw, group=group, deep=deep, schedule=sched)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        slow = max(times)
        res[n] = {"shard_ms": [round(t * 1e3, 2) for t in times],
                  "kernel_ms": {abi.KERNEL_NAMES[i]: round(st.kernel_ms[i], 2) for i in range(abi.XRT_K_COUNT)
                                if st.kernel_ms[i]},
                  "msamples_s": round(W * H * SPP / slow / 1e6, 1), "iterations": int(st.iterations),
                  "schedule": abi.SCHEDULE_NAMES[st.schedule]}
        print(n, res[n], flush=True)
    print(json.dumps({"config": cfg_name, "shards": res}))
    r.close()


if __name__ == "__main__":
    main()
