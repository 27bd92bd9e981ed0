"""bench.py --gpus N: the launch plan is decided before any GPU call and never
renders N > 1 GPUs' worth of work on one GPU — torchrun's WORLD_SIZE must equal N, a bare
`--gpus N` on a node with N GPUs starts N ranks itself, and too few GPUs is an error."""
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
