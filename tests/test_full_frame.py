"""Full-frame parity at the benchmark configurations (C3, C4), every pixel.

* C3 (Conference 1920x1080, 1 spp, Whitted): all 2,058,240 primary hit ids (kind, input index,
  t bits) and the whole bitmap bit-exact against the oracle; rows 1072-1079 untouched.
* C4 (1920x1080, 4 spp, PathTracer, depth 5): the whole bitmap bit-exact, the ray count equal.
* Cull invariance at full size: no cull / fast cull / certified cull give the same bitmap, hits
  and ray counts.
* Random rays through the whole room: closest hits and shadow tests of 4M rays, every cull mode
  against the reference walk, and a sample against the oracle.

The scene is the Conference stand-in (mobileraytracer_amd/scenes.py: the real conference.obj is
absent from the reference snapshot).
"""
import os

import numpy as np
import pytest

from test_gpu_parity import SENTINEL, make_cfg, oracle_for

pytestmark = pytest.mark.gpu

THREADS = 16  # the GPU box's CPU share


def oracle_full(oracle_mod, cfg):
    o = oracle_for(oracle_mod, cfg)
    bm = np.full(cfg.width * cfg.height, SENTINEL, np.int32)
    _, rays = o.render(bm, threads=THREADS)
    o.close()
    return bm, rays


@pytest.fixture(scope="module")
def c3_gpu():
    import mobileraytracer_amd as m
    cfg = make_cfg(1920, 1080, shader=1, scene="conference")
    out = {}
    with m.Renderer(cfg) as r:
        for cull in (1, 0, 2, 3):
            r.set_tuning(2, cull)
            bm = np.full(1920 * 1080, SENTINEL, np.int32)
            r.render_frame(bm)
            out[cull] = (bm, r.frame_stats(), r.primary_hits())
    return cfg, out


def test_c3_primary_hits_full_frame(oracle_mod, c3_gpu):
    cfg, out = c3_gpu
    o = oracle_for(oracle_mod, cfg)
    ok, oi, ot = o.primary_hits()
    o.close()
    k, i, t = out[3][2]  # the default (exact) mode
    rendered = ok >= 0
    assert rendered.sum() == 1920 * 1072
    assert np.array_equal(k, ok) and np.array_equal(i, oi)
    assert np.array_equal(t.view(np.int32), ot.view(np.int32))
    assert (k[rendered] > 0).mean() > 0.99  # the room is closed: nearly every camera ray hits


def test_c3_whitted_bitmap_full_frame(oracle_mod, c3_gpu):
    cfg, out = c3_gpu
    bm, st, _ = out[3]
    ref, ref_rays = oracle_full(oracle_mod, cfg)
    rows = bm.reshape(1080, 1920)
    assert (rows[1072:] == SENTINEL).all()  # H / 16 = 67: rows 1072-1079 never rendered (Renderer.cpp:33-34)
    assert (rows[:1072] != SENTINEL).all()
    assert np.array_equal(bm, ref), int((bm != ref).sum())
    assert st["rays"] + st["shadowRays"] == ref_rays


def test_c3_cull_modes_identical_full_frame(c3_gpu):
    _, out = c3_gpu
    base_bm, base_st, base_hits = out[3]
    for cull in (0, 1, 2):
        bm, st, hits = out[cull]
        assert np.array_equal(bm, base_bm), cull
        assert (st["rays"], st["shadowRays"]) == (base_st["rays"], base_st["shadowRays"])
        assert all(np.array_equal(a, b) for a, b in zip(hits, base_hits))


@pytest.fixture(scope="module")
def c4_gpu():
    import mobileraytracer_amd as m
    cfg = make_cfg(1920, 1080, shader=2, scene="conference", spp=4, max_depth=5)
    out = {}
    with m.Renderer(cfg) as r:
        for cull in (1, 0, 2, 3):
            r.set_tuning(2, cull)
            bm = np.full(1920 * 1080, SENTINEL, np.int32)
            r.render_frame(bm)
            out[cull] = (bm, r.frame_stats())
    return cfg, out


def test_c4_pathtracer_full_frame(oracle_mod, c4_gpu):
    cfg, out = c4_gpu
    bm, st = out[3]
    assert st["primaryRays"] == 4 * 1920 * 1072
    ref, ref_rays = oracle_full(oracle_mod, cfg)
    assert np.array_equal(bm, ref), int((bm != ref).sum())
    assert st["rays"] + st["shadowRays"] == ref_rays


def test_c4_cull_modes_identical_full_frame(c4_gpu):
    _, out = c4_gpu
    base_bm, base_st = out[3]
    for cull in (0, 1, 2):
        bm, st = out[cull]
        assert np.array_equal(bm, base_bm), (cull, int((bm != base_bm).sum()))
        assert (st["rays"], st["shadowRays"]) == (base_st["rays"], base_st["shadowRays"])


def random_rays(n, seed, box_min, box_max):
    rng = np.random.default_rng(seed)
    o = (box_min + rng.random((n, 3)) * (box_max - box_min)).astype(np.float32)
    d = rng.normal(size=(n, 3))
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    return o, d


def test_random_rays_all_cull_modes(oracle_mod):
    """4M rays from random points of the room in random directions, closest hit and a shadow test
    to a random distance: walk 1 in every cull mode equals the reference walk (walk 0), and a
    20,000-ray sample equals the oracle."""
    import mobileraytracer_amd as m
    cfg = make_cfg(64, 64, shader=1, scene="conference")
    with m.Renderer(cfg) as r:
        boxes, _, _, _ = m.triangle_bvh(cfg)
        lo, hi = boxes[0, :3], boxes[0, 3:]
        o, d = random_rays(4_000_000, 7, lo, hi)
        dist = np.random.default_rng(8).random(len(o)).astype(np.float32) * np.float32(np.linalg.norm(hi - lo))
        res = {}
        for walk, cull in ((0, 0), (1, 0), (1, 1), (1, 2), (1, 3)):
            r.set_tuning(1, walk)
            r.set_tuning(2, cull)
            res[(walk, cull)] = (r.trace_rays(o, d), r.trace_rays(o, d, dist=dist, any_hit=True)[0])
    ref_hits, ref_occ = res[(0, 0)]
    assert (ref_hits[0] == 3).mean() > 0.5 and 0.05 < ref_occ.mean() < 0.95
    for key, (hits, occ) in res.items():
        assert all(np.array_equal(a, b) for a, b in zip(hits, ref_hits)), key
        assert np.array_equal(occ, ref_occ), key
    o_ = oracle_for(oracle_mod, cfg)
    sel = np.arange(0, len(o), len(o) // 20000)
    ok, oi, ot = o_.trace_rays(o[sel], d[sel])
    occ = o_.trace_rays(o[sel], d[sel], dist=dist[sel], any_hit=True)[0]
    o_.close()
    assert np.array_equal(ok, ref_hits[0][sel]) and np.array_equal(oi, ref_hits[1][sel])
    assert np.array_equal(ot.view(np.int32), ref_hits[2][sel].view(np.int32))
    assert np.array_equal(occ, ref_occ[sel])


@pytest.mark.parametrize("scene", ["conference", "water"])
def test_walk_tree_rays_with_zero_direction_components(oracle_mod, scene):
    """The walk tree regroups the reference leaves (rebuildOverLeaves); it reaches exactly the
    reference's triangles for rays with a finite 1/d (leaf-box reachability).
    Rays with a zero direction component (1/d infinite, NaN slabs on box faces) walk the reference
    tree instead.  Both kinds, from random points and from points ON box planes (where the
    reference's NaN order decides), equal the oracle: closest hit and shadow test."""
    import mobileraytracer_amd as m
    cfg = make_cfg(64, 64, shader=1, scene=scene)
    boxes, _, _, _ = m.triangle_bvh(cfg)
    lo, hi = boxes[0, :3], boxes[0, 3:]
    rng = np.random.default_rng(5)
    n = 30000
    o, d = random_rays(n, 3, lo, hi)
    d = d.copy()
    k = n // 3
    d[:k, rng.integers(0, 3)] = 0.0                      # one zero component
    d[k:2 * k:2, :] = 0.0
    d[k:2 * k:2, rng.integers(0, 3)] = rng.choice([-1.0, 1.0])  # axis-aligned
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    leaf = boxes[np.any(boxes != 0, axis=1)]
    pick = leaf[rng.integers(0, len(leaf), k)]
    o[2 * k:, :] = pick[: n - 2 * k, :3]               # origins on box min corners (NaN slabs)
    dist = (rng.random(n) * np.linalg.norm(hi - lo)).astype(np.float32)
    with m.Renderer(cfg) as r:
        hits = r.trace_rays(o, d)
        occ = r.trace_rays(o, d, dist=dist, any_hit=True)[0]
    ob = oracle_for(oracle_mod, cfg)
    ok, oi, ot = ob.trace_rays(o, d)
    oocc = ob.trace_rays(o, d, dist=dist, any_hit=True)[0]
    ob.close()
    assert np.array_equal(hits[0], ok) and np.array_equal(hits[1], oi)
    assert np.array_equal(hits[2].view(np.int32), ot.view(np.int32))
    assert np.array_equal(occ, oocc)


def test_walk_tree_is_invariant():
    """C4-style frames with the regrouped walk tree (default) and with the reference tree as the
    walk tree (MOBILERT_WALK_TREE=0): identical bitmaps and ray counts."""
    import os
    import mobileraytracer_amd as m
    outs = []
    for env in ("0", "1"):
        os.environ["MOBILERT_WALK_TREE"] = env
        try:
            cfg = make_cfg(320, 192, shader=2, scene="conference", spp=2, max_depth=5)
            with m.Renderer(cfg) as r:
                bm = np.zeros(cfg.width * cfg.height, np.int32)
                r.render_frame(bm)
                st = r.frame_stats()
                outs.append((bm, st["rays"], st["shadowRays"]))
        finally:
            del os.environ["MOBILERT_WALK_TREE"]
    assert np.array_equal(outs[0][0], outs[1][0]) and outs[0][1:] == outs[1][1:]


def test_quantized_walk_tree_boundary_rays(oracle_mod):
    """The walk tree's boxes are 16-bit grid coordinates rounded outward by one step, under an
    error bound that holds for 1/d components in [2^-40, 2^90] and origins within 4 grid extents
    (DESIGN.md section 3.1); walk-tree leaves are tested exactly.  Rays built to sit on that
    argument's edges - aimed at leaf-box corners, edges and faces (tangent to exact leaf boxes),
    starting on leaf-box faces, with direction components of 1e-27 / 1e-29 (1/d just inside /
    outside 2^90), from 3.9 and 4.1 grid extents away - give the reference walk's closest hits and
    shadow tests in every cull mode, and a sample equals the oracle."""
    import mobileraytracer_amd as m
    cfg = make_cfg(64, 64, shader=1, scene="conference")
    boxes, off, cnt, _ = m.triangle_bvh(cfg)
    lo, hi = boxes[0, :3].astype(np.float64), boxes[0, 3:].astype(np.float64)
    ext = hi - lo
    leaf = boxes[cnt > 0].astype(np.float64)
    rng = np.random.default_rng(11)
    parts = []
    n = 200_000
    # aimed at a corner / an edge point / a face point of a random leaf box
    o, _ = random_rays(3 * n, 12, lo, hi)
    o = o.astype(np.float64)
    b = leaf[rng.integers(0, len(leaf), 3 * n)]
    t = b[:, :3] + rng.random((3 * n, 3)) * (b[:, 3:] - b[:, :3])
    corner = np.where(rng.random((3 * n, 3)) < 0.5, b[:, :3], b[:, 3:])
    t[:n] = corner[:n]                                   # corners
    ax = rng.integers(0, 3, (3 * n, 2))
    idx = np.arange(3 * n)
    t[n:2 * n, :][np.arange(n), ax[n:2 * n, 0]] = corner[n:2 * n][np.arange(n), ax[n:2 * n, 0]]
    t[n:2 * n, :][np.arange(n), ax[n:2 * n, 1]] = corner[n:2 * n][np.arange(n), ax[n:2 * n, 1]]  # edges
    t[2 * n:, :][np.arange(n), ax[2 * n:, 0]] = corner[2 * n:][np.arange(n), ax[2 * n:, 0]]      # faces
    parts.append((o, t - o))
    # starting on a leaf-box face, random directions
    o2 = leaf[rng.integers(0, len(leaf), n)]
    p = o2[:, :3] + rng.random((n, 3)) * (o2[:, 3:] - o2[:, :3])
    a = rng.integers(0, 3, n)
    p[np.arange(n), a] = np.where(rng.random(n) < 0.5, o2[np.arange(n), a], o2[np.arange(n), 3 + a])
    parts.append((p, rng.normal(size=(n, 3))))
    # tiny direction components around the 2^90 bound on 1/d, and far origins around 4 extents
    k = 20_000
    o3, d3 = random_rays(k, 13, lo, hi)
    d3 = d3.astype(np.float64)
    d3[: k // 2, rng.integers(0, 3)] = rng.choice([1e-27, -1e-27])
    d3[k // 2:, rng.integers(0, 3)] = rng.choice([1e-29, -1e-29])
    parts.append((o3.astype(np.float64), d3))
    c = (lo + hi) / 2
    for f in (3.9, 4.1):
        dirn = rng.normal(size=(k, 3))
        dirn /= np.linalg.norm(dirn, axis=1, keepdims=True)
        far = c - dirn * (f * ext.max() + np.linalg.norm(ext))
        tgt = lo + rng.random((k, 3)) * ext
        parts.append((far, tgt - far))
    o = np.concatenate([q[0] for q in parts]).astype(np.float32)
    d = np.concatenate([q[1] for q in parts])
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    dist = (rng.random(len(o)) * np.linalg.norm(ext) * 2).astype(np.float32)
    res = {}
    with m.Renderer(cfg) as r:
        for walk, cull in ((0, 0), (1, 0), (1, 1), (1, 2), (1, 3)):
            r.set_tuning(1, walk)
            r.set_tuning(2, cull)
            res[(walk, cull)] = (r.trace_rays(o, d), r.trace_rays(o, d, dist=dist, any_hit=True)[0])
    ref_hits, ref_occ = res[(0, 0)]
    assert (ref_hits[0] == 3).mean() > 0.3
    for key, (hits, occ) in res.items():
        assert all(np.array_equal(x, y) for x, y in zip(hits, ref_hits)), key
        assert np.array_equal(occ, ref_occ), key
    o_ = oracle_for(oracle_mod, cfg)
    sel = np.concatenate([np.arange(0, 4 * n, 100), np.arange(4 * n, len(o), 10)])
    ok, oi, ot = o_.trace_rays(o[sel], d[sel])
    occ = o_.trace_rays(o[sel], d[sel], dist=dist[sel], any_hit=True)[0]
    o_.close()
    assert np.array_equal(ok, ref_hits[0][sel]) and np.array_equal(oi, ref_hits[1][sel])
    assert np.array_equal(ot.view(np.int32), ref_hits[2][sel].view(np.int32))
    assert np.array_equal(occ, ref_occ[sel])


def test_packet_walk_grazing_bundles(oracle_mod):
    """The camera rays' packet walk (tuning key 16) enters a child when ANY walking lane passes its
    quantized box and orders children by the first walking lane's entry, then each lane tests the
    exact reference leaf box, the certified leaf key and its own triangles.  Its hits equal the
    per-lane walk's provided every quantized ancestor box holds the exact box of every leaf below it
    as the slab test computes it (the Quantizer's margin).  Coherent 64-ray
    bundles (one packet each: mrt_trace_rays fills waves with 64 consecutive rays) aimed tangent
    to leaf-box corners, edges and faces, with a spread of 1e-7 .. 1e-3 rad, stress exactly that:
    packet on / off and cull modes 0 / 3 give the reference walk's hits, and a sample the oracle's."""
    import mobileraytracer_amd as m
    cfg = make_cfg(64, 64, shader=1, scene="conference")
    boxes, off, cnt, _ = m.triangle_bvh(cfg)
    lo, hi = boxes[0, :3].astype(np.float64), boxes[0, 3:].astype(np.float64)
    leaf = boxes[cnt > 0].astype(np.float64)
    rng = np.random.default_rng(21)
    nb = 4096  # bundles
    b = leaf[rng.integers(0, len(leaf), nb)]
    corner = np.where(rng.random((nb, 3)) < 0.5, b[:, :3], b[:, 3:])
    tgt = b[:, :3] + rng.random((nb, 3)) * (b[:, 3:] - b[:, :3])
    kind = rng.integers(0, 3, nb)  # 0 corner, 1 edge, 2 face
    ax = rng.integers(0, 3, (nb, 2))
    for i in range(nb):
        if kind[i] == 0:
            tgt[i] = corner[i]
        else:
            tgt[i, ax[i, 0]] = corner[i, ax[i, 0]]
            if kind[i] == 1:
                tgt[i, ax[i, 1]] = corner[i, ax[i, 1]]
    o = lo + rng.random((nb, 3)) * (hi - lo)
    d0 = tgt - o
    d0 /= np.linalg.norm(d0, axis=1, keepdims=True)
    spread = 10.0 ** rng.uniform(-7, -3, nb)
    jit = rng.normal(size=(nb, 64, 3)) * spread[:, None, None]
    jit[:, 0] = 0.0  # the bundle's first ray exactly at the target
    d = d0[:, None, :] + jit
    d = (d / np.linalg.norm(d, axis=2, keepdims=True)).reshape(-1, 3).astype(np.float32)
    o = np.repeat(o, 64, axis=0).astype(np.float32)
    res = {}
    with m.Renderer(cfg) as r:
        for walk, cull, packet in ((0, 0, 0), (1, 3, 1), (1, 3, 0), (1, 0, 1), (1, 0, 0)):
            r.set_tuning(1, walk)
            r.set_tuning(2, cull)
            r.set_tuning(16, packet)
            res[(walk, cull, packet)] = r.trace_rays(o, d)
    ref = res[(0, 0, 0)]
    assert (ref[0] == 3).mean() > 0.5
    for key, hits in res.items():
        assert all(np.array_equal(x, y) for x, y in zip(hits, ref)), key
    o_ = oracle_for(oracle_mod, cfg)
    sel = np.arange(0, len(o), 37)
    ok, oi, ot = o_.trace_rays(o[sel], d[sel])
    o_.close()
    assert np.array_equal(ok, ref[0][sel]) and np.array_equal(oi, ref[1][sel])
    assert np.array_equal(ot.view(np.int32), ref[2][sel].view(np.int32))


# ---- the flat-geometry stand-in (scenes.conference_flat): large flat triangles, slivers, abutting
# and overlapping coplanar panels - the shapes that stress the certified leaf key, the quantized
# walk tree's margins and the exact-t tie rule at full frame
@pytest.fixture(scope="module")
def c3_flat():
    import mobileraytracer_amd as m
    cfg = make_cfg(1920, 1080, shader=1, scene="conference_flat")
    out = {}
    with m.Renderer(cfg) as r:
        for cull in (3, 0, 1):
            r.set_tuning(2, cull)
            bm = np.full(1920 * 1080, SENTINEL, np.int32)
            r.render_frame(bm)
            out[cull] = (bm, r.frame_stats(), r.primary_hits())
    return cfg, out


def test_flat_c3_primary_hits_and_bitmap_full_frame(oracle_mod, c3_flat):
    cfg, out = c3_flat
    bm, st, (k, i, t) = out[3]
    o = oracle_for(oracle_mod, cfg)
    ok, oi, ot = o.primary_hits()
    o.close()
    assert (ok >= 0).sum() == 1920 * 1072
    assert np.array_equal(k, ok) and np.array_equal(i, oi)
    assert np.array_equal(t.view(np.int32), ot.view(np.int32))
    ref, ref_rays = oracle_full(oracle_mod, cfg)
    assert np.array_equal(bm, ref), int((bm != ref).sum())
    assert st["rays"] + st["shadowRays"] == ref_rays
    for cull in (0,):  # no cull: the reference's visit set, the same image
        assert np.array_equal(out[cull][0], bm) and all(np.array_equal(a, b) for a, b in zip(out[cull][2], out[3][2]))


def test_flat_c4_pathtracer_full_frame(oracle_mod):
    import mobileraytracer_amd as m
    cfg = make_cfg(1920, 1080, shader=2, scene="conference_flat", spp=4, max_depth=5)
    outs = {}
    with m.Renderer(cfg) as r:
        for cull in (3, 0):
            r.set_tuning(2, cull)
            bm = np.full(1920 * 1080, SENTINEL, np.int32)
            r.render_frame(bm)
            outs[cull] = (bm, r.frame_stats())
    bm, st = outs[3]
    assert st["primaryRays"] == 4 * 1920 * 1072
    ref, ref_rays = oracle_full(oracle_mod, cfg)
    assert np.array_equal(bm, ref), int((bm != ref).sum())
    assert st["rays"] + st["shadowRays"] == ref_rays
    assert np.array_equal(outs[0][0], bm)


def test_flat_grazing_rays_along_surfaces(oracle_mod):
    """Rays starting ON the flat stand-in's triangles (walls, floor panels, table, paper sheets,
    slivers) and leaving at 1e-6 .. 1e-2 rad from their plane, with the triangle as the source
    primitive (self-exclusion, Triangle.cpp:64-66): the grazing, nearly coplanar case in which
    Moller-Trumbore's t can fall before a triangle's box entry.  Closest hit and shadow test equal
    the reference walk in every cull mode except the documented inexact one, and a sample the oracle."""
    import mobileraytracer_amd as m
    cfg = make_cfg(64, 64, shader=1, scene="conference_flat")
    from mobileraytracer_amd import scenes
    obj = scenes.conference_flat()[0]
    verts, faces = [], []
    with open(obj) as f:
        for line in f:
            if line.startswith("v "):
                verts.append([float(x) for x in line.split()[1:4]])
            elif line.startswith("f "):
                faces.append([int(x) - 1 for x in line.split()[1:4]])
    V = np.asarray(verts, np.float64)
    V[:, 0] = -V[:, 0]  # the loader negates X (OBJLoader.cpp:139-141)
    F = np.asarray(faces)[:-2]  # the last two faces are the light panel
    rng = np.random.default_rng(31)
    n = 200_000
    pick = rng.integers(0, len(F), n)
    A, B, C = V[F[pick, 0]], V[F[pick, 1]], V[F[pick, 2]]
    w = rng.random((n, 2))
    w[w.sum(1) > 1] = 1 - w[w.sum(1) > 1]
    o = A + w[:, :1] * (B - A) + w[:, 1:] * (C - A)
    nrm = np.cross(B - A, C - A)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    tang = rng.normal(size=(n, 3))
    tang -= (tang * nrm).sum(1, keepdims=True) * nrm
    tang /= np.linalg.norm(tang, axis=1, keepdims=True)
    ang = 10.0 ** rng.uniform(-6, -2, n) * rng.choice([-1.0, 1.0], n)
    d = tang * np.cos(ang)[:, None] + nrm * np.sin(ang)[:, None]
    o32, d32 = o.astype(np.float32), (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    src = np.stack([np.full(n, 3), pick], 1).astype(np.int32)  # (kind triangle, input index)
    dist = (rng.random(n) * 3000.0).astype(np.float32)
    res = {}
    with m.Renderer(cfg) as r:
        for walk, cull in ((0, 0), (1, 0), (1, 2), (1, 3)):
            r.set_tuning(1, walk)
            r.set_tuning(2, cull)
            res[(walk, cull)] = (r.trace_rays(o32, d32, src=src), r.trace_rays(o32, d32, dist=dist, src=src, any_hit=True)[0])
    ref_hits, ref_occ = res[(0, 0)]
    assert (ref_hits[0] == 3).mean() > 0.5
    for key, (hits, occ) in res.items():
        assert all(np.array_equal(x, y) for x, y in zip(hits, ref_hits)), key
        assert np.array_equal(occ, ref_occ), key
    ob = oracle_for(oracle_mod, cfg)
    sel = np.arange(0, n, 20)
    ok, oi, ot = ob.trace_rays(o32[sel], d32[sel], src=src[sel])
    oocc = ob.trace_rays(o32[sel], d32[sel], dist=dist[sel], src=src[sel], any_hit=True)[0]
    ob.close()
    assert np.array_equal(ok, ref_hits[0][sel]) and np.array_equal(oi, ref_hits[1][sel])
    assert np.array_equal(ot.view(np.int32), ref_hits[2][sel].view(np.int32))
    assert np.array_equal(oocc, ref_occ[sel])
