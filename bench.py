"""bench.py — BASELINE.json metric: Msamples/s (whole node) + wall-clock at 800x600x1024 spp.

One step = one full frame of the workload (default C2: Cornell box 800x600, 1024 spp,
GIIntegrator(3)), rendered by the MI355X wavefront through libxrt_hip.so with the scene
already resident in HBM.  With N GPUs (one process per GPU) each rank renders the rows
y % N == rank and rank 0 assembles the frame with one RCCL gather of every rank's packed rows
(--assembly reduce: a SUM reduce of the zero-elsewhere framebuffers; both exact).  Total work
is fixed as N grows: "strong".  Under torchrun
WORLD_SIZE must equal N; without a launcher and N > 1 the bench starts N ranks itself
(torch.distributed.run, child process); it exits non-zero rather than render N > 1 on one GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2] [--no-cpu]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Msamples/s (whole node) + wall-clock at 800×600×1024spp, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3        # vector FP32 spec
# VALU issue peak: 256 CUs x 4 SIMD-32 units, a wave64 vector instruction issues over 2
# cycles (MI355X_MICROARCH.md: "issues each VALU instruction over 2 cycles"), 2.4 GHz max
# clock -> 1,024 * 2.4e9 / 2 = 1,228.8 G wave-instructions/s (= the FP32 vector peak / 128)
SIMDS, CLOCK_HZ, VALU_CYCLES = 1024, 2.4e9, 2
VALU_PEAK_GINST = SIMDS * CLOCK_HZ / VALU_CYCLES / 1e9

# Roofline model: algorithmic bytes per sample of the
# path, B_s = 68 + 264·Q + 12·D, with Q = extension segments per sample and D = RNG draws
# per sample (both counted by the device and identical to the CPU restatement's counts):
#   68  per sample  — 44 B generated ray (o, d, thr, pixel, depth) + 24 B accumulate RMW
#   264 per segment — extend (o,d read 24 + hit write 16), shade (read 44 + 16, write next
#                     ray 44 + shadow ray 44), shadow (read 44 + RMW 24), compaction 8
#   12  per draw    — 4 B tempered word + 8 B amortised twist (2 * 2496 B / 624)
# The fused schedule (k_step / k_step_tri) performs all of it in one kernel; the wavefront
# schedule splits it: k_trace = extend + shadow (108·Q), k_shade = the rest.
B_SAMPLE, B_SEGMENT, B_DRAW = 68, 264, 12
B_TRACE_SEG = 24 + 16 + 44 + 24
# k_pixel (Direct / Normal pixel chains) never writes path records; what it must move is each
# pixel's seeded mt19937 state (624 words, read once) and its framebuffer pixel (read + write)
PIX_STATE_BYTES = 624 * 4
FLOP_PER_TRI_TEST = 40          # Moller-Trumbore arithmetic per triangle test (secondary)


def env_int(k, d):
    try:
        return int(os.environ.get(k, d))
    except ValueError:
        return d


def cpu_quota():
    """CPUs the cgroup lets this process use (cpu.max quota / period), or None."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(p)
    except (OSError, ValueError):
        return None


# Bounded CPU sample per workload (about 10-20 s of the oracle on the box's 16 CPUs): rows
# y % shard_count == 0 of the workload's own image at `spp` samples per pixel.  The oracle
# restates the reference's linear scans (no acceleration structure), so C3's 1,001 spheres
# and C4's 51,236 triangles cost far more per sample than C2's 36 triangles.
CPU_SAMPLE = {"C1": (1, 256), "C2": (1, 256), "C3": (4, 96), "C4": (256, 2), "C5": (1, 512)}


def cpu_baseline(cfg_name, cfg, spp=None):
    """The oracle (CPU restatement, bit-exact with the GPU path) on every CPU this process
    may use: one OpenMP thread per CPU of os.sched_getaffinity, or per CPU of the cgroup's
    CPU quota when that is smaller (more threads than the quota only time-slice: measured
    7.3 Msamples/s with 256 threads under a 16-CPU quota, 10.7 with 16)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from xraytracer_amd import scenes
    affinity = max(1, len(os.sched_getaffinity(0)))
    quota = cpu_quota()
    threads = affinity if not quota else max(1, min(affinity, int(quota + 0.5)))
    shards, dspp = CPU_SAMPLE.get(cfg_name, (1, 256))
    spp = spp or dspp
    s = scenes.build(cfg_name)
    w, h = cfg["width"], cfg["height"]
    t0 = time.perf_counter()
    _, st = pyoracle.render(s, w, h, spp, nthreads=threads, shard_index=0, shard_count=shards)
    dt = time.perf_counter() - t0
    rows = len(range(0, h, shards))
    what = f"rows y % {shards} == 0 ({rows} of {h}) of " if shards > 1 else ""
    return {"value": round(st["samples"] / dt / 1e6, 6), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{what}{cfg_name} scene {w}x{h} at {spp} spp ({st['samples']} samples; cost is linear in "
                      f"spp), oracle/oracle.c (the reference's linear scans) with OpenMP over rows, {threads} threads "
                      f"= every CPU this process may use ({affinity} in its affinity mask"
                      + (f", cgroup CPU quota {quota:g}" if quota else "") + f"), {dt:.2f} s wall"}


def plan_launch(gpus, env, device_count):
    """How `bench.py --gpus N` runs (decided before any GPU call):
    ("run", world)  — this process is one rank of `world` (torchrun set WORLD_SIZE = N, or N = 1);
    ("spawn", N)    — no launcher and N > 1: start N ranks with torch.distributed.run as a child
                      process on this node and exit with its status;
    ("error", msg)  — N disagrees with WORLD_SIZE, or the node has fewer than N GPUs.
    It never renders N > 1 on one GPU.  device_count: torch.cuda.device_count() (counting does
    not initialise the GPU on this image)."""
    if gpus < 1:
        return ("error", f"--gpus must be >= 1, got {gpus}")
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        try:
            world = int(ws)
        except ValueError:
            return ("error", f"WORLD_SIZE={ws!r} is not an integer")
        if world != gpus:
            return ("error", f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
        local = int(env.get("LOCAL_RANK", "0"))
        if local >= device_count:
            return ("error", f"LOCAL_RANK {local} but only {device_count} GPU(s) visible")
        return ("run", world)
    if gpus > device_count:
        return ("error", f"--gpus {gpus} but only {device_count} GPU(s) visible")
    return ("run", 1) if gpus == 1 else ("spawn", gpus)


def spawn_ranks(n, argv):
    """One rank per GPU via torch.distributed.run (child process; this process never touched
    the GPU).  Returns the launcher's exit status."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def hip_kernel_name(kid, sched, scene):
    """The HIP kernel behind an xrt_stats kernel family for this schedule / scene (the name
    rocprofv3 reports, which the PMC summaries are keyed by)."""
    from xraytracer_amd import abi
    if kid == abi.XRT_K_STEP:
        if sched == abi.XRT_SCHED_PIXEL:
            return "k_pixel"
        if sched in (abi.XRT_SCHED_STEP_MERGED, abi.XRT_SCHED_STEP_BVH):   # k_step_merged<..., BVH>
            return "k_step_merged"
        return "k_step_tri" if sched == abi.XRT_SCHED_STEP_TRI else "k_step"
    if kid == abi.XRT_K_TRACE and scene.desc.n_tris > 1024:   # two-level trace: phase A
        return "k_trace_2a_coop"
    return "k_" + abi.KERNEL_NAMES[kid]


def load_keyed(path, cfg, kernel):
    """A PMC / traffic summary (tools/prof_summary.py) if it is for this config and kernel."""
    try:
        j = json.load(open(path))
    except (OSError, ValueError):
        return None
    return j if j.get("config") == cfg and j.get("kernel") == kernel else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--spp", type=int, default=None, help="override spp (never for reported numbers)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-spp", type=int, default=None, help="override the CPU sample's spp")
    ap.add_argument("--no-timing", action="store_true", help="skip per-kernel HIP events")
    ap.add_argument("--schedule", default="auto", choices=("auto", "step", "wavefront"))
    ap.add_argument("--traffic", default=None, help="default profiles/traffic_<CONFIG>.json")
    ap.add_argument("--pmc", default=None, help="default profiles/pmc_<CONFIG>.json")
    ap.add_argument("--no-spec", action="store_true", help="no speculative sample starts (XRT_FLAG_NO_SPEC)")
    ap.add_argument("--assembly", default="gather", choices=("gather", "reduce"),
                    help="N > 1: frame assembly on rank 0 — gather each rank's owned rows, or reduce(SUM) full frames")
    ap.add_argument("--test-standin", default=None, metavar="MODULE:FACTORY",
                    help="TESTS ONLY (tests/test_bench_launch.py): a CPU stand-in renderer instead of the HIP one")
    args = ap.parse_args()
    args.traffic = args.traffic or os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
    args.pmc = args.pmc or os.path.join(ROOT, "profiles", f"pmc_{args.config}.json")

    import numpy as np
    import torch

    # Tests only (tests/test_bench_launch.py): --test-standin MODULE:FACTORY swaps the HIP
    # renderer for a CPU stand-in (not the oracle) so the multi-rank plumbing — the spawn,
    # torch.distributed.run's rank environment, process-group init, the frame assembly and the
    # max-over-ranks timing — runs end to end on a GPU-less machine over gloo.  An explicit
    # flag (forwarded to the spawned ranks with the rest of argv), announced on stderr, and a
    # stand-in line says so in "data".
    standin = args.test_standin
    if standin:
        print(f"bench.py: WARNING: --test-standin {standin}: CPU stand-in renderer, not a measurement",
              file=sys.stderr, flush=True)
    on_gpu = not standin
    devices = torch.cuda.device_count() if on_gpu else env_int("XRT_BENCH_STANDIN_DEVICES", 8)
    action, what = plan_launch(args.gpus, os.environ, devices)
    if action == "error":
        print(f"bench.py: {what}", file=sys.stderr, flush=True)
        sys.exit(2)
    if action == "spawn":
        sys.exit(spawn_ranks(what, sys.argv[1:]))

    from xraytracer_amd import abi, distributed, scenes
    from xraytracer_amd.renderer import HipRenderer

    world = what
    rank = env_int("RANK", 0)
    local = env_int("LOCAL_RANK", 0)
    dist = None
    if world > 1:
        import datetime
        import torch.distributed as dist
        # an explicit collective timeout: a rank that never arrives ends the job instead of
        # hanging it (XRT_DIST_TIMEOUT_S, default 10 minutes)
        timeout = datetime.timedelta(seconds=env_int("XRT_DIST_TIMEOUT_S", 600))
        if on_gpu:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout)
        else:
            dist.init_process_group("gloo", timeout=timeout)
    elif on_gpu:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local) if on_gpu else torch.device("cpu")

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    cfg = dict(scenes.CONFIGS[args.config])
    if args.spp:
        cfg["spp"] = args.spp
    W, H, SPP = cfg["width"], cfg["height"], cfg["spp"]
    scene = scenes.build(args.config)
    if standin:
        import importlib
        mod, fn = standin.split(":")
        r = getattr(importlib.import_module(mod), fn)(SPP, local)
    else:
        r = HipRenderer(SPP, device=local)
    r.upload(scene)
    fb = torch.zeros((H, W, 3), dtype=torch.float32, device=dev)
    timing = not args.no_timing

    sharded = distributed.ShardedRenderer(r, dist, time_reduce=True, assembly=args.assembly)

    def step(timed):
        # rank's rows, then the frame assembled on rank 0 (gather of the owned rows, or a
        # reduce(SUM)); the render waits for the work queued on torch's stream (the previous
        # step's collective) before it overwrites fb
        return sharded.render(scene, W, H, fb, timing=timing and timed, schedule=args.schedule,
                              **({"spec": False} if args.no_spec else {}))

    for _ in range(args.warmup):
        step(False)
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    agg = {k: 0.0 for k in ("segments", "shadow_rays", "draws", "samples", "iterations", "rejected")}
    kms = np.zeros(abi.XRT_K_COUNT)
    kl = np.zeros(abi.XRT_K_COUNT)
    reduce_s = 0.0
    for _ in range(args.steps):
        st = step(True)
        reduce_s += sharded.last_reduce_s
        for k in agg:
            agg[k] += getattr(st, k)
        kms += np.array(list(st.kernel_ms))
        sched = int(st.schedule)
        kl += np.array(list(st.launches))
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        elapsed = distributed.max_over_ranks(elapsed, dist, device=dev)
        reduce_s = distributed.max_over_ranks(reduce_s, dist, device=dev)
        agg = distributed.sum_counters(agg, dist, device=dev)

    if rank == 0:
        total_samples = W * H * SPP * args.steps
        value = total_samples / elapsed / 1e6
        ms = elapsed / args.steps * 1e3
        # roofline of the dominant kernel (per-launch algorithmic bytes / avg launch time)
        roof = None
        if timing and kms.sum() > 0:
            samples = agg["samples"] / max(1, world)            # this rank's share
            q = agg["segments"] / max(1, agg["samples"])
            dpp = agg["draws"] / max(1, agg["samples"])
            b_s = B_SAMPLE + B_SEGMENT * q + B_DRAW * dpp
            dom = max((abi.XRT_K_TRACE, abi.XRT_K_SHADE, abi.XRT_K_STEP, abi.XRT_K_DEEP), key=lambda k: kms[k])
            if dom == abi.XRT_K_STEP:
                kbytes = b_s * samples
            elif dom == abi.XRT_K_TRACE:
                kbytes = B_TRACE_SEG * q * samples
            elif dom == abi.XRT_K_SHADE:
                kbytes = (b_s - B_TRACE_SEG * q) * samples
            else:   # the deep BVH walk: only its queued rays' share of the trace is known per ray
                kbytes = None
            launches = max(1, kl[dom])
            avg_s = kms[dom] / 1e3 / launches
            kname = hip_kernel_name(dom, sched, scene)
            # measured traffic and limiter, from the PMC passes of the same kernel and workload
            # (tools/evidence.sh CONFIG -> tools/prof_summary.py -> profiles/{pmc,traffic}_CONFIG.json):
            #   VALU issue: SQ_INSTS_VALU per launch / avg launch time vs VALU_PEAK_GINST
            #   HBM:        (FETCH_SIZE x2 + WRITE_SIZE) per launch / avg launch time vs 8 TB/s
            tj = load_keyed(args.traffic, args.config, kname)
            traffic = tj.get("hbm_bytes_per_launch") if tj else None
            pmc = load_keyed(args.pmc, args.config, kname)
            model = None
            if sched == abi.XRT_SCHED_PIXEL:
                # k_pixel keeps a pixel's whole sample chain in registers and LDS: the bytes it
                # needs are each pixel's seeded mt19937 state (read once) and its framebuffer
                # pixel (read, written); the scene is read into LDS per block (L2-resident)
                kbytes = samples / SPP * (PIX_STATE_BYTES + 24)
                per_launch = kbytes / launches
                achieved = per_launch / avg_s / 1e9
                model = {"what": "k_pixel required bytes: seeded mt19937 state 2,496 B + framebuffer read/write "
                                 "24 B per pixel",
                         "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "bytes_per_pixel": PIX_STATE_BYTES + 24,
                         "algorithmic_bytes_per_launch": round(per_launch, 1),
                         "soa_model_not_applicable": "SURVEY.md 8d's B_s = 68 + 264*Q + 12*D prices the SoA "
                                                     "wavefront form of the path (ray, hit and shadow records "
                                                     "per segment); k_pixel writes none of them"}
            elif kbytes is not None:
                per_launch = kbytes / launches
                achieved = per_launch / avg_s / 1e9
                model = {"what": "SURVEY.md 8d algorithmic bytes, B_s = 68 + 264*Q + 12*D per sample",
                         "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "bytes_per_sample": round(b_s, 2),
                         "algorithmic_bytes_per_launch": round(per_launch, 1)}
                if model["frac"] > 1.0:
                    # the fused kernels keep path state on chip: the model's bytes are those of
                    # the SoA wavefront form of the path, not a bound on this kernel
                    model["applicable"] = False
                    model["note"] = ("not applicable (frac > 1): the kernel keeps the path state the model streams "
                                     "in registers / LDS; hbm_measured is what it moves")
            hbm = None
            if traffic:
                hbm = {"achieved": round(traffic / avg_s / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": round(traffic / avg_s / 1e9 / HBM_PEAK_GBS, 5), "bytes_per_launch": traffic}
            valu = None
            if pmc and pmc.get("SQ_INSTS_VALU_per_launch"):
                vi = pmc["SQ_INSTS_VALU_per_launch"]
                valu = {"achieved": round(vi / avg_s / 1e9, 2), "peak": round(VALU_PEAK_GINST, 1),
                        "unit": "Gwave-inst/s", "frac": round(vi / avg_s / 1e9 / VALU_PEAK_GINST, 5),
                        "valu_insts_per_launch": vi,
                        "valu_insts_per_sample": round(vi * kl[dom] / max(1.0, samples), 2),
                        "lane_utilisation": pmc.get("lane_utilisation"),
                        "valu_active_per_wave_cycle": pmc.get("valu_active_per_wave_cycle"),
                        "wait_per_wave_cycle": pmc.get("wait_per_wave_cycle")}
            if valu and (not hbm or valu["frac"] >= hbm["frac"]):
                head, bound = valu, "valu"
            elif hbm:
                head, bound = hbm, "hbm"
            elif model and model.get("applicable", True):   # no counters: the model figure, labelled as such
                head, bound = model, "hbm (model; unmeasured)"
            else:
                head, bound = {"achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None}, "unmeasured"
            roof = {"bound": bound, "kernel": kname, "achieved": head["achieved"], "peak": head["peak"],
                    "unit": head["unit"], "frac": head["frac"], "traffic": traffic,
                    "traffic_source": (tj or {}).get("source"),
                    "avg_launch_us": round(avg_s * 1e6, 3), "launches": int(kl[dom]),
                    "valu_issue": valu, "hbm_measured": hbm, "model": model,
                    "pmc_source": (pmc or {}).get("source")}
            # secondary: the reference's brute-force triangle tests (every object, every
            # triangle; shadow rays skip area-light objects) x FLOP_PER_TRI_TEST — only for
            # the small triangle scenes whose traces are (culled) linear scans
            d = scene.desc
            n_occ = sum(d.objects[i].count for i in range(d.n_objects)
                        if d.objects[i].kind == abi.XRT_OBJ_MESH and d.objects[i].light < 0)
            tests = (agg["segments"] * d.n_tris + agg["shadow_rays"] * n_occ) / max(1, world)
            if tests and d.n_tris <= 1024:   # linear scans only (larger scenes trace a BVH)
                tf = tests * FLOP_PER_TRI_TEST / (kms[dom] / 1e3) / 1e12
                roof["valu"] = {"tri_tests_per_sample": round(tests / max(1, samples), 2),
                                "achieved_tflops": round(tf, 3), "peak_tflops": FP32_PEAK_TFLOPS,
                                "frac": round(tf / FP32_PEAK_TFLOPS, 4)}
            roof["kernel_ms_per_step"] = {abi.KERNEL_NAMES[i]: round(kms[i] / args.steps, 3)
                                          for i in range(abi.XRT_K_COUNT) if kms[i]}
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic" if on_gpu else f"STAND-IN renderer {standin} (plumbing test, not a measurement)",
            "config": {"workload": f"{args.config}: {cfg['scene']} {W}x{H}, {SPP} spp, {cfg['integrator']}"
                                   f"(maxDepth={cfg['max_depth']})",
                       "width": W, "height": H, "spp": SPP, "integrator": cfg["integrator"],
                       "max_depth": cfg["max_depth"], "global_batch": W * H * SPP,
                       "parallelism": (f"pixel rows y%{world} per GPU + RCCL {args.assembly} to rank 0" if world > 1
                                       else "1 GPU"),
                       "segments_per_sample": round(agg["segments"] / max(1, agg["samples"]), 4),
                       "draws_per_sample": round(agg["draws"] / max(1, agg["samples"]), 4),
                       "iterations_per_frame": round(agg["iterations"] / args.steps, 1),
                       "schedule": abi.SCHEDULE_NAMES[sched],
                       "shadow_rays_per_sample": round(agg["shadow_rays"] / max(1, agg["samples"]), 4)},
            "roofline": roof,
            "cpu_baseline": None,
        }
        if world > 1:   # the RCCL frame assembly, inside ms_per_step (slowest rank)
            out["config"]["assembly"] = args.assembly
            out["config"]["assembly_ms_per_step"] = round(reduce_s / args.steps * 1e3, 3)
            out["config"]["assembly_bytes"] = distributed.assembly_bytes(H, W, world, args.assembly)
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(args.config, cfg, args.cpu_spp)
        print(json.dumps(out), flush=True)
    r.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
