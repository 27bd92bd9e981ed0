"""bench.py --gpus N: the launch plan is decided before any GPU call and never
renders N > 1 GPUs' worth of work on one GPU — torchrun's WORLD_SIZE must equal N, a bare
`--gpus N` on a node with N GPUs starts N ranks itself, and too few GPUs is an error."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


@pytest.mark.parametrize("gpus,env,devs,expect", [
    (1, {}, 1, ("run", 1)),
    (1, {}, 8, ("run", 1)),
    (8, {}, 8, ("spawn", 8)),
    (2, {}, 8, ("spawn", 2)),
    (8, {"WORLD_SIZE": "8", "LOCAL_RANK": "7"}, 8, ("run", 8)),
    (2, {"WORLD_SIZE": "2", "LOCAL_RANK": "0"}, 8, ("run", 2)),
    (1, {"WORLD_SIZE": "1", "LOCAL_RANK": "0"}, 1, ("run", 1)),
])
def test_plan_runs_or_spawns(gpus, env, devs, expect):
    assert bench.plan_launch(gpus, env, devs) == expect


@pytest.mark.parametrize("gpus,env,devs", [
    (2, {}, 1),                                         # fewer GPUs than asked: never one GPU
    (8, {}, 0),
    (1, {}, 0),
    (2, {"WORLD_SIZE": "4", "LOCAL_RANK": "0"}, 8),     # launcher and --gpus disagree
    (8, {"WORLD_SIZE": "1", "LOCAL_RANK": "0"}, 8),
    (4, {"WORLD_SIZE": "4", "LOCAL_RANK": "3"}, 2),     # rank without a device
    (0, {}, 8),
    (2, {"WORLD_SIZE": "two"}, 8),
])
def test_plan_errors(gpus, env, devs):
    assert bench.plan_launch(gpus, env, devs)[0] == "error"


def test_bench_exits_nonzero_without_enough_gpus():
    """The real entry point on this GPU-less container: `--gpus 2` must fail, not print a
    1-GPU line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-cpu"],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode != 0
    assert '"n_gpus"' not in r.stdout
    assert "GPU" in r.stderr


def _standin_env(tmp_path, **extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env["HIP_VISIBLE_DEVICES"] = ""
    env["XRT_BENCH_STANDIN_DEVICES"] = "2"
    env["XRT_BENCH_STANDIN_OUT"] = str(tmp_path / "frames")
    env["XRT_DIST_TIMEOUT_S"] = "60"
    env["PYTHONPATH"] = os.path.join(ROOT, "tests") + os.pathsep + env.get("PYTHONPATH", "")
    env.update(extra)
    return env


def test_bench_spawns_two_ranks_end_to_end(tmp_path):
    """`bench.py --gpus 2` without a launcher, end to end on CPU — plan_launch,
    spawn_ranks' torch.distributed.run child, the rank environment, process-group init (gloo
    with the stand-in renderer; nccl = RCCL on the GPU node), ShardedRenderer's row shards and
    framebuffer reduce, the max-over-ranks timing and the whole-job counters: rank 0 prints
    exactly one n_gpus 2 line carrying assembly_ms_per_step, and both ranks rendered every step."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-cpu", "--config", "C1",
                        "--steps", "3", "--warmup", "1", "--no-timing", "--test-standin", "bench_standin:make"],
                       capture_output=True, text=True, env=_standin_env(tmp_path), timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = lines[0]
    assert d["n_gpus"] == 2 and d["steps"] == 3 and "STAND-IN" in d["data"]
    assert d["config"]["assembly"] == "gather" and d["config"]["assembly_ms_per_step"] >= 0
    assert d["config"]["assembly_bytes"] == 128 * 256 * 3 * 4   # rank 1's 128 packed rows
    assert "--test-standin" in r.stderr
    assert d["config"]["parallelism"].startswith("pixel rows y%2")
    assert d["config"]["segments_per_sample"] == 1.0 and d["config"]["draws_per_sample"] == 2.0   # summed over ranks
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # warmup + 3 timed steps on every rank; rank 0 found the whole frame (every row y holding
    # y + 1 from the rank that owns it) after each of the first three reduces
    assert open(tmp_path / "frames.0").read() == "4 3"
    assert open(tmp_path / "frames.1").read().split()[0] == "4"


def test_bench_failing_rank_fails_the_job(tmp_path):
    """A rank that raises ends the job with a non-zero status and no bench line."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-cpu", "--config", "C1",
                        "--steps", "2", "--warmup", "0", "--no-timing", "--test-standin", "bench_standin:make"],
                       capture_output=True, text=True, env=_standin_env(tmp_path, XRT_BENCH_STANDIN_FAIL_RANK="1"),
                       timeout=300)
    assert r.returncode != 0
    assert '"n_gpus"' not in r.stdout
    assert "fails on purpose" in r.stderr
