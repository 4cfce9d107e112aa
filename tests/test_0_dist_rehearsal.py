"""Multi-rank rehearsal of bench.py's distributed path.

bench.py under torch.distributed.run, and `bench.py --gpus 2` spawning its own ranks, with 2 ranks on the one GPU of a test box: the gloo
backend (MRT_BENCH_BACKEND=gloo: the gather goes through host memory; the measured multi-GPU path
is RCCL with one GPU per rank), each rank renders its screen-tile shard into a packed buffer,
rank 0 gathers and unpacks.  Rank 0's assembled bitmap must equal the single-GPU bench's and the
oracle's.  The file name sorts first so that this test starts its child processes before the
pytest process itself initialises the GPU (no process may exec another after that).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

W, H, SPP = 320, 192, 4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench(tmp, name, nproc, launcher=True, extra_env=None, extra_args=()):
    out = os.path.join(tmp, name + ".npy")
    args = ["bench.py", "--gpus", str(nproc), "--steps", "1", "--warmup", "0", "--no-cpu-baseline",
            "--width", str(W), "--height", str(H), "--spp", str(SPP), "--dump-bitmap", out] + list(extra_args)
    env = dict(os.environ, MRT_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    env.update(extra_env or {})
    if nproc > 1 and launcher:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
    else:
        cmd = [sys.executable] + args
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    return np.load(out), line


def test_two_rank_bench_assembles_the_single_gpu_frame(tmp_path, oracle_mod):
    import json
    import torch
    assert not torch.cuda.is_initialized(), "must run before this process touches the GPU"
    two, line2 = _bench(str(tmp_path), "two", 2)
    one, _ = _bench(str(tmp_path), "one", 1)
    j = json.loads(line2)
    assert j["n_gpus"] == 2 and "gloo gather" in j["config"]["parallelism"]
    assert np.array_equal(two, one), int((two != one).sum())
    from mobileraytracer_amd import scenes
    obj, mtl, cam = scenes.conference()
    o = oracle_mod.Oracle(W, H, 2, -1, SPP, 1, 5, obj=obj, mtl=mtl, cam=cam)
    ref = np.zeros(W * H, np.int32)
    o.render(ref, threads=min(16, os.cpu_count() or 1))
    o.close()
    assert np.array_equal(two, ref), int((two != ref).sum())
    # the driver's form: `python bench.py --gpus 2` with no launcher spawns its own 2 ranks
    spawned, line_s = _bench(str(tmp_path), "spawned", 2, launcher=False)
    js = json.loads(line_s)
    assert js["n_gpus"] == 2 and "gloo gather" in js["config"]["parallelism"]
    assert np.array_equal(spawned, one), int((spawned != one).sum())
    # the RCCL path itself at world size 1 (MRT_BENCH_FORCE_DIST: process group, packed shard,
    # gather, unpack) assembles the same frame
    rccl = dict(MRT_BENCH_BACKEND="nccl", MRT_BENCH_FORCE_DIST="1", RANK="0", LOCAL_RANK="0", WORLD_SIZE="1",
                MASTER_PORT=str(_free_port()))
    img, line_r = _bench(str(tmp_path), "rccl", 1, launcher=False, extra_env=rccl,
                         extra_args=("--steps", "3", "--warmup", "2"))
    jr = json.loads(line_r)
    assert "RCCL gather" in jr["config"]["parallelism"], jr["config"]["parallelism"]
    assert np.array_equal(img, one), int((img != one).sum())


def test_group_bench_assembles_the_single_gpu_frame(tmp_path):
    """`bench.py --gpus 4 --path group`: the front ends' multi-GPU path (one process, one Renderer
    over a device group, MOBILERT_DEVICES) with the ordinal repeated on the one-GPU box; the
    assembled bitmap equals the single-GPU bench's frame."""
    import json
    import torch
    assert not torch.cuda.is_initialized(), "must run before this process touches the GPU"
    one, _ = _bench(str(tmp_path), "one_g", 1)
    grp, line = _bench(str(tmp_path), "group", 4, launcher=False, extra_env={"MOBILERT_DEVICES": "0,0,0,0"},
                       extra_args=("--path", "group", "--steps", "2", "--warmup", "1"))
    j = json.loads(line)
    assert j["n_gpus"] == 4 and j["config"]["parallelism"].startswith("device group x4"), j["config"]
    assert j["config"]["devices"] == [0, 0, 0, 0]
    assert j["value"] > 0 and j["roofline"]["kernels"]["k_trace"]["avg_launch_ms"] > 0
    assert np.array_equal(grp, one), int((grp != one).sum())


def test_distinct_gpus_rccl_and_group_bench(tmp_path):
    """Where the box has several GPUs: bench.py's RCCL rank path (one GPU per rank, `--gpus 2`
    spawning its ranks) and its device-group path over distinct ordinals (peer copies) assemble the
    single-GPU frame.  Skipped on one-GPU boxes, where the rehearsals above stand in for them."""
    import json
    import torch
    n = torch.cuda.device_count()  # (counting devices does not initialise them)
    if n < 2:
        pytest.skip("one visible GPU: distinct-device paths need two")
    assert not torch.cuda.is_initialized(), "must run before this process touches the GPU"
    one, _ = _bench(str(tmp_path), "one_d", 1)
    rccl, line = _bench(str(tmp_path), "rccl2", 2, launcher=False, extra_env={"MRT_BENCH_BACKEND": "nccl"})
    assert "RCCL gather" in json.loads(line)["config"]["parallelism"]
    assert np.array_equal(rccl, one), int((rccl != one).sum())
    k = min(8, n)
    grp, line = _bench(str(tmp_path), "group_d", k, launcher=False, extra_env={"MOBILERT_DEVICES": ""},
                       extra_args=("--path", "group"))
    j = json.loads(line)
    assert j["config"]["devices"] == list(range(k)) and j["n_gpus"] == k
    assert np.array_equal(grp, one), int((grp != one).sum())
