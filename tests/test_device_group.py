"""Device groups: one frame sharded over several GPUs through the C-ABI the front ends call.

The reference's Renderer::renderFrame spreads one frame over all its workers
(app/MobileRT/Renderer.cpp:62-82; RayTrace times it, C_wrapper.cpp:227-236).  mrt_config.devices
(MOBILERT_DEVICES for RayTrace, the Android session and the C++ facade) does the same over GPUs:
shard i of the screen-tile partition renders on devices[i] from a host thread of its own, and the
head (devices[0]) gathers the packed shards (peer copies) and unpacks the frame.  On the one-GPU
test box the ordinals repeat (0,0,0,0): the shards then share the GPU, which exercises every step
of the group path except the xGMI transfer itself.  On a box with several GPUs the same checks
also run with distinct ordinals (0,1 and every visible GPU up to 8): the peer-access setup and the
hipMemcpyPeerAsync assembly.  The bitmap, getSample() and getTotalCastedRays() must equal the
single-GPU renderer's bit for bit.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO
from test_gpu_parity import SENTINEL, make_cfg

pytestmark = pytest.mark.gpu

CASES = (
    dict(width=320, height=192, shader=2, scene="conference", spp=4, max_depth=5),
    dict(width=128, height=128, shader=1, scene="water", max_depth=4),
    dict(width=96, height=96, shader=2, scene="water", spp=2, spl=3, max_depth=4),
    dict(width=128, height=128, shader=2, scene="teapot", spp=2, max_depth=3),
    dict(width=64, height=64, shader=2, spp=3, max_depth=6),
    dict(width=80, height=48, shader=3, scene="water"),
)


def _device_lists():
    """Repeated ordinals always; distinct ones where the box has several GPUs."""
    import torch
    n = torch.cuda.device_count()  # (counting devices does not initialise them)
    lists = [[0, 0], [0, 0, 0, 0]]
    if n >= 2:
        lists += [[0, 1], list(range(min(8, n)))]
    return lists


def _render(cfg, frames=1):
    import mobileraytracer_amd as m
    with m.Renderer(cfg) as r:
        out = []
        for _ in range(frames):
            bm = np.full(cfg.width * cfg.height, SENTINEL, np.int32)
            r.render_frame(bm)
            st = r.frame_stats()
            out.append((bm, r.get_sample(), r.get_total_casted_rays(), st["rays"], st["shadowRays"], st["walkedRays"]))
        return out, r.scene_info()


@pytest.mark.parametrize("idx", range(len(CASES)))
@pytest.mark.parametrize("progressive", (0, 1))
def test_device_group_equals_single_gpu(idx, progressive):
    kw = dict(CASES[idx])
    single, _ = _render(make_cfg(**kw, progressive=progressive), frames=2)
    for devices in _device_lists():
        group, info = _render(make_cfg(**kw, progressive=progressive, devices=devices), frames=2)
        assert info["deviceCount"] == len(devices)
        for a, b in zip(single, group):
            assert np.array_equal(a[0], b[0]), (devices, int((a[0] != b[0]).sum()))
            assert a[1:] == b[1:], (devices, a[1:], b[1:])


def test_device_group_device_path_primary_hits_and_stop():
    import torch
    import mobileraytracer_amd as m
    kw = dict(width=160, height=96, shader=2, scene="conference", spp=2, max_depth=5)
    ref = _render(make_cfg(**kw))[0][0][0]
    with m.Renderer(make_cfg(**kw)) as r:
        hk, hi, ht = r.primary_hits()
    with m.Renderer(make_cfg(**kw, devices=[0, 0, 0])) as g:
        # into device memory on devices[0], on the caller's stream
        d = torch.full((kw["width"] * kw["height"],), int(SENTINEL), dtype=torch.int32, device="cuda")
        g.render_frame_device(d.data_ptr(), 0, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy(), ref)
        with pytest.raises(Exception):  # a group assembles its own frame: no packed output
            g.render_frame_device(0, d.data_ptr(), 0)
        k, i, t = g.primary_hits()
        assert np.array_equal(k, hk) and np.array_equal(i, hi) and np.array_equal(t.view(np.int32), ht.view(np.int32))
        # tuning reaches every shard: same frame with the shadow walks serialised
        g.set_tuning(3, 0)
        bm = np.full(kw["width"] * kw["height"], SENTINEL, np.int32)
        g.render_frame(bm)
        assert np.array_equal(bm, ref)
        # stopRender reaches every shard: nothing more is rendered, getSample() stays 0
        g.stop_render()
        bm = np.full(kw["width"] * kw["height"], SENTINEL, np.int32)
        g.render_frame(bm)
        assert (bm == SENTINEL).all() and g.get_sample() == 0


def test_device_group_rejects_bad_configs():
    import mobileraytracer_amd as m
    with pytest.raises(Exception):
        m.Renderer(make_cfg(64, 64, devices=[0, 999]))
    with pytest.raises(Exception):
        m.Renderer(make_cfg(64, 64, devices=[0, 0], rankCount=2))


def test_raytrace_and_facade_with_mobilert_devices(tmp_path):
    """RayTrace(Config&, bool) and the C++ MobileRT::Renderer facade with MOBILERT_DEVICES=0,0,0:
    every bitmap, getSample() and getTotalCastedRays() equal the single-GPU run's."""
    from mobileraytracer_amd import scenes
    runs = {}
    import torch
    groups = [("group", "0,0,0")] + ([("group_distinct", "0,1")] if torch.cuda.device_count() >= 2 else [])
    for name, devs in [("single", None)] + groups:
        env = dict(os.environ)
        env.pop("MOBILERT_MAX_DEPTH", None)
        env.pop("MOBILERT_DEVICES", None)
        if devs:
            env["MOBILERT_DEVICES"] = devs
        d1, d2 = tmp_path / (name + "_cabi"), tmp_path / (name + "_facade")
        d1.mkdir()
        d2.mkdir()
        p = subprocess.run([os.path.join(REPO, "tests", "cabi", "build", "raytrace_cabi"), str(d1),
                            *scenes.cornell_water()], capture_output=True, text=True, timeout=240, env=env)
        assert p.returncode == 0, p.stdout + p.stderr
        q = subprocess.run([os.path.join(REPO, "tests", "cabi", "build", "renderer_facade"), str(d2),
                            *scenes.cornell_water(), *scenes.teapot()], capture_output=True, text=True, timeout=240,
                           env=env)
        assert q.returncode == 0, q.stdout + q.stderr
        runs[name] = (d1, d2, [l for l in p.stdout.splitlines() if l.startswith("Casted rays")])
    s1, s2, srays = runs["single"]
    for name, _ in groups:
        g1, g2, grays = runs[name]
        assert srays == grays and srays
        for d, e in ((s1, g1), (s2, g2)):
            names = sorted(f for f in os.listdir(d) if f != "async_stop.bin")  # async_stop: a partial frame
            assert names and names == sorted(f for f in os.listdir(e) if f != "async_stop.bin")
            for f in names:
                assert open(d / f, "rb").read() == open(e / f, "rb").read(), (name, f)
