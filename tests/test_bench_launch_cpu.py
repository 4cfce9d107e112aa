"""bench.py --gpus N: how the process decides to run, spawn N ranks or refuse (CPU only).

The driver runs `python bench.py --gpus N` with or without torch.distributed.run; both must run N
ranks, one GPU each, and a mismatch must fail loudly before anything touches the GPU."""
import os
import subprocess
import sys

from conftest import REPO

sys.path.insert(0, REPO)
from bench import launch_plan  # noqa: E402


def test_single_gpu_runs_in_process():
    assert launch_plan(1, {}, 1) == ("run", None)
    assert launch_plan(1, {}, 0) == ("run", None)  # the renderer itself fails loudly without a GPU


def test_n_gpus_without_launcher_spawns_n_ranks():
    assert launch_plan(8, {}, 8) == ("spawn", 8)
    assert launch_plan(2, {"MRT_BENCH_BACKEND": "gloo"}, 1) == ("spawn", 2)  # rehearsal: ranks share a GPU


def test_more_ranks_than_gpus_is_refused():
    act, msg = launch_plan(8, {}, 1)
    assert act == "error" and "8" in msg and "1 visible" in msg
    act, msg = launch_plan(4, {"WORLD_SIZE": "4", "LOCAL_WORLD_SIZE": "4"}, 2)
    assert act == "error" and "one GPU per rank" in msg


def test_launcher_world_must_equal_gpus():
    assert launch_plan(2, {"WORLD_SIZE": "2", "LOCAL_WORLD_SIZE": "2"}, 8) == ("run", None)
    act, msg = launch_plan(8, {"WORLD_SIZE": "2"}, 8)
    assert act == "error" and "WORLD_SIZE=2" in msg
    act, msg = launch_plan(1, {"WORLD_SIZE": "4"}, 8)
    assert act == "error"


def test_bad_count_is_refused():
    assert launch_plan(0, {}, 8)[0] == "error"


def test_cli_refuses_before_touching_a_gpu():
    # this container has no GPU: --gpus 3 over RCCL must exit 2 with the message, not start ranks
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MRT_BENCH_BACKEND")}
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "3", "--steps", "1"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2, (p.returncode, p.stderr[-2000:])
    assert "one GPU per rank" in p.stderr
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=REPO, env=dict(env, WORLD_SIZE="3"),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2 and "WORLD_SIZE=3" in p.stderr, p.stderr[-2000:]


def test_group_path_runs_in_one_process():
    from bench import group_devices
    # --path group: one process for the whole device group, never spawned
    assert launch_plan(4, {}, 4, "group") == ("run", None)
    assert launch_plan(4, {"MOBILERT_DEVICES": "0,0,0,0"}, 1, "group") == ("run", None)  # one-GPU rehearsal
    assert group_devices(3, {}) == [0, 1, 2]
    assert group_devices(4, {"MOBILERT_DEVICES": "0,0,0,0"}) == [0, 0, 0, 0]


def test_group_path_refuses_bad_device_lists():
    act, msg = launch_plan(4, {}, 2, "group")
    assert act == "error" and "2 visible" in msg
    act, msg = launch_plan(4, {"MOBILERT_DEVICES": "0,0"}, 1, "group")
    assert act == "error" and "lists 2" in msg
    act, msg = launch_plan(2, {"MOBILERT_DEVICES": "0,1x"}, 8, "group")
    assert act == "error" and "bad ordinal '1x'" in msg
    act, msg = launch_plan(2, {"MOBILERT_DEVICES": "0,-1"}, 8, "group")
    assert act == "error" and "bad ordinal" in msg
    act, msg = launch_plan(2, {"WORLD_SIZE": "2"}, 8, "group")
    assert act == "error" and "without a launcher" in msg
