"""Pins the CPU oracle against the reference's own known-answer tests (app/Unit_Testing/*.cpp,
scripts/test/docker/dockerfile.sh) before it is trusted as the parity oracle.  CPU only."""
import os

import numpy as np
import pytest

F = np.float32


def ulp_eq(a, b, ulps=4):
    """gtest ASSERT_FLOAT_EQ: within 4 ULPs."""
    a, b = F(a), F(b)
    ia, ib = np.array([a]).view(np.int32)[0], np.array([b]).view(np.int32)[0]
    if ia < 0:
        ia = np.int32(-2 ** 31) - ia
    if ib < 0:
        ib = np.int32(-2 ** 31) - ib
    return abs(int(ia) - int(ib)) <= ulps


def sub(a, b):
    return tuple(F(x) - F(y) for x, y in zip(a, b))


# ---- TestTriangle.cpp:347-433 (triangle A(0,0,0) B(0,1,0) C(0,0,1)) -----------------------
TRI = ((0, 0, 0), (0, 1, 0), (0, 0, 1))


@pytest.mark.parametrize("orig,target,expected", [
    ((2, 0, 0), (0, 0, 0), True),            # intersectRayInside01
    ((2, 0, 0), (0, 1, 0), True),            # intersectRayInside02
    ((2, 0, 0), (0, 0, 1), True),            # intersectRayInside03
    ((2, 0, 0), (0, 1.000001, 0), False),    # intersectRayOutside01
    ((2, 0, 0), (0, 0, 1.000001), False),    # intersectRayOutside02
    ((2, 2, 2), (0.000001, 0, 0), False),    # intersectRayOutside03
    ((2, 2, 2), (-1, 0, 0), False),          # intersectRayOutside04
    ((2, 0, 0), (0, -0.000001, 0), False),   # intersectRayOutside05
    ((2, 0, 0), (0, 0, -0.000001), False),   # intersectRayOutside06
])
def test_triangle_ray_kat(oracle_mod, orig, target, expected):
    hit, _ = oracle_mod.kat_triangle(*TRI, orig, sub(target, orig))
    assert hit == expected


def test_triangle_self_exclusion_kat(oracle_mod):  # intersectRayFromPrimitive
    hit, _ = oracle_mod.kat_triangle(*TRI, (2, 0, 0), sub((0, 0, 0), (2, 0, 0)), from_self=True)
    assert not hit


def test_triangle_aabb_kat(oracle_mod):  # TestTriangle.cpp:206-216
    mn, mx = oracle_mod.triangle_aabb(*TRI)
    assert mn == (0.0, 0.0, 0.0) and mx == (0.0, 1.0, 1.0)


# ---- TestAABB.cpp:51-130 ------------------------------------------------------------------
def test_aabb_centroid_area_kat(oracle_mod):
    c, a = oracle_mod.aabb_props((0, 0, 0), (1, 0, 0))
    assert c == (0.5, 0.0, 0.0) and a == 0.0
    _, a2 = oracle_mod.aabb_props((0, 0, 0), (1, 1, 0))
    assert a2 == 2.0


def test_aabb_ray_kat_nan_path(oracle_mod):
    # zero-thickness box, direction components 0 on axes 1-2: (0-0)*inf = NaN there, which the
    # libstdc++ min/max operand order ignores
    assert oracle_mod.kat_aabb((0, 0, 0), (1, 0, 0), (2, 0, 0), (-1, 0, 0)) is True
    assert oracle_mod.kat_aabb((0, 0, 0), (1, 0, 0), (2, 0, 0), (1, 0, 0)) is False


def test_aabb_nan_on_axis0_misses(oracle_mod):
    # NaN produced on axis 0 poisons tMin/tMax -> miss (the asymmetric half of Appendix A.3)
    assert oracle_mod.kat_aabb((0, 0, 0), (0, 1, 1), (0, 0.5, 2), (0, 0, -1)) is False


# ---- TestPlane.cpp:239-281 ----------------------------------------------------------------
def test_plane_aabb_kat(oracle_mod):
    mn, mx = oracle_mod.plane_aabb((-1, 0, 0), (1, 0, 0))
    exp_mn, exp_mx = (-1, -70.7107, -70.7107), (-1, 70.7107, 70.7107)
    assert all(ulp_eq(a, b) for a, b in zip(mn, exp_mn))
    assert all(ulp_eq(a, b) for a, b in zip(mx, exp_mx))


def test_plane_ray_kat(oracle_mod):
    hit, _ = oracle_mod.kat_plane((-1, 0, 0), (1, 0, 0), (0, 0, 10), (10, 0, 10))
    assert not hit  # IntersectionRayOutsideX
    hit, t = oracle_mod.kat_plane((-1, 0, 0), (1, 0, 0), (0, 0, 10), (-10, 0, 10))
    assert hit and t == pytest.approx(0.1)  # IntersectionRayInsideX


# ---- TestRay.cpp:54-63 ------------------------------------------------------------------------
def test_ray_id_kat(oracle_mod):
    assert oracle_mod.lib().oracle_kat_ray_ids() == 1


# ---- TestCameraLoader.cpp:19-49 ---------------------------------------------------------------
def test_camera_loader_kat(oracle_mod, tmp_path):
    p = tmp_path / "c.cam"
    p.write_text("\nt perspective\np 0 30.0 -200.0\nl 0.0 30.0 100.0\nu 0.0 1.0 0.0\nf 44 45\n    ")
    c = oracle_mod.kat_camera(str(p), 1.0)
    for got, exp in zip(c["position"] + c["direction"] + c["up"], (0, 30, -200, 0, 0, 1, 0, 1, 0)):
        assert ulp_eq(got, exp)
    assert ulp_eq(c["hfov"], 44.0) and ulp_eq(c["vfov"], 45.0)


# ---- loader KATs: scripts/test/docker/dockerfile.sh:118-119 + resource fixtures -----------------
def test_scene_counts_kat(oracle_mod):
    from mobileraytracer_amd import scenes
    o = oracle_mod.Oracle(32, 32, 1, -1, obj=scenes.cornell_water()[0], mtl=scenes.cornell_water()[1],
                          cam=scenes.cornell_water()[2])
    c = o.counts()
    assert c["triangles"] + c["lights"] == 7088 and c["lights"] == 2
    obj, mtl, cam = scenes.conference()
    o = oracle_mod.Oracle(32, 32, 1, -1, obj=obj, mtl=mtl, cam=cam)
    c = o.counts()
    assert c["triangles"] == scenes.CONFERENCE_TRIANGLES and c["lights"] == scenes.CONFERENCE_LIGHTS


def test_conference_camera(oracle_mod):
    from mobileraytracer_amd import scenes
    c = oracle_mod.kat_camera(scenes.conference()[2], np.float32(1920) / np.float32(1080))
    assert c["position"] == [460.0, 500.0, -1000.0]  # X negated (PerspectiveLoader.cpp:52)
    assert c["hfov"] == pytest.approx(80.0, rel=1e-6) and c["vfov"] == pytest.approx(45.0, rel=1e-6)


# ---- numerics (Utils.cpp, Perspective.cpp, libstdc++ partition) ------------------------------
def test_halton_kat(oracle_mod):
    assert [oracle_mod.halton(i) for i in range(8)] == [0, 0.5, 0.25, 0.75, 0.125, 0.625, 0.375, 0.875]
    t = oracle_mod.table(0x4D525401)  # a permutation of {k / 2^20}
    assert np.array_equal(np.sort(t.astype(np.float64) * (1 << 20)), np.arange(1 << 20, dtype=np.float64))


def test_incremental_avg_kat(oracle_mod):
    assert oracle_mod.incremental_avg((1.0, 1.0, 1.0), 0, 1) == -1  # 0xFFFFFFFF
    first = oracle_mod.incremental_avg((0.5, 0.25, 0.0), 0, 1)
    assert first == np.int32(np.uint32(0xFF000000 | 0 << 16 | 63 << 8 | 127))
    second = oracle_mod.incremental_avg((1.0, 0.0, 2.0), first, 2)
    # R (127+255)/2 = 191, G (63+0)/2 = 31, B (0+510)/2 = 255
    assert second == np.int32(np.uint32(0xFF000000 | 255 << 16 | 31 << 8 | 191))


def test_fast_arctan(oracle_mod):
    assert oracle_mod.fast_arctan(1.0) == np.float32(np.pi / 4)
    assert oracle_mod.fast_arctan(0.0) == 0.0


def test_partition_matches_libstdcxx(oracle_mod):
    assert oracle_mod.selftest_partition(7, 3000) == 0


def test_sample_streams_are_pure(oracle_mod):
    k = oracle_mod.path_key(1234, 3)
    assert k == oracle_mod.path_key(1234, 3) and k != oracle_mod.path_key(1234, 2)
    idx = {oracle_mod.sample_index(k, 1, p) for p in range(16)}
    assert len(idx) == 16 and max(idx) < (1 << 20)
