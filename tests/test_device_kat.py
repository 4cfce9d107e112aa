"""Device known-answer tests: the slab and triangle tests the trace kernels inline
(mrt_device.hpp slab / slabFinite / triTest), run by a tiny HIP kernel (mrt_kat_slab,
mrt_kat_triangle) on the reference's own unit-test vectors and compared with the oracle.

* TestTriangle.cpp:347-433: hit / miss at +-1e-6 of the triangle's edges and vertices;
* TestAABB.cpp:111-130: a zero-thickness box hit along its extent, i.e. 0 * inf = NaN on axes
  1-2, which the libstdc++ std::min / std::max operand order ignores;
* the axis-0 NaN case (poisons tMin / tMax: a miss) and random boxes / rays (both slab forms).
"""
import numpy as np
import pytest

from test_oracle_kat import TRI, sub

pytestmark = pytest.mark.gpu

F = np.float32

TRI_CASES = [
    ((2, 0, 0), (0, 0, 0), True),            # intersectRayInside01
    ((2, 0, 0), (0, 1, 0), True),            # intersectRayInside02
    ((2, 0, 0), (0, 0, 1), True),            # intersectRayInside03
    ((2, 0, 0), (0, 1.000001, 0), False),    # intersectRayOutside01
    ((2, 0, 0), (0, 0, 1.000001), False),    # intersectRayOutside02
    ((2, 2, 2), (0.000001, 0, 0), False),    # intersectRayOutside03
    ((2, 2, 2), (-1, 0, 0), False),          # intersectRayOutside04
    ((2, 0, 0), (0, -0.000001, 0), False),   # intersectRayOutside05
    ((2, 0, 0), (0, 0, -0.000001), False),   # intersectRayOutside06
]


def test_triangle_kat_on_device(oracle_mod):
    import mobileraytracer_amd as m
    tris = np.array([np.array(TRI, F).ravel() for _ in TRI_CASES], F)
    orig = np.array([c[0] for c in TRI_CASES], F)
    dirs = np.array([sub(c[1], c[0]) for c in TRI_CASES], F)
    hit, t = m.kat_triangle(tris, orig, dirs)
    assert hit.tolist() == [int(c[2]) for c in TRI_CASES]
    for k, (o, tgt, _) in enumerate(TRI_CASES):
        ohit, ot = oracle_mod.kat_triangle(*TRI, o, sub(tgt, o))
        assert bool(hit[k]) == ohit
        if ohit:
            assert np.float32(t[k]).view(np.int32) == np.float32(ot).view(np.int32)


def test_slab_kat_nan_paths_on_device(oracle_mod):
    import mobileraytracer_amd as m
    cases = [  # (min, max, origin, direction, expected) - TestAABB.cpp:111-130 and Appendix A.3
        ((0, 0, 0), (1, 0, 0), (2, 0, 0), (-1, 0, 0), True),    # NaN on axes 1-2: ignored
        ((0, 0, 0), (1, 0, 0), (2, 0, 0), (1, 0, 0), False),
        ((0, 0, 0), (0, 1, 1), (0, 0.5, 2), (0, 0, -1), False),  # NaN on axis 0: miss
        ((0, 0, 0), (1, 1, 1), (0.5, 0.5, -3), (0, 0, 1), True),  # inf 1/d on axes 0-1, finite box
    ]
    boxes = np.array([c[0] + c[1] for c in cases], F)
    orig = np.array([c[2] for c in cases], F)
    dirs = np.array([c[3] for c in cases], F)
    out = m.kat_slab(boxes, orig, dirs)
    assert out[:, 0].tolist() == [int(c[4]) for c in cases]
    for k, c in enumerate(cases):
        assert bool(out[k, 0]) == oracle_mod.kat_aabb(c[0], c[1], c[2], c[3])
    assert out[:, 2].tolist() == [0, 0, 0, 0]  # every case has a zero direction component


def test_slab_forms_agree_on_random_boxes(oracle_mod):
    """The IEEE min/max form the kernels use for rays with finite 1/d returns the reference
    predicate on 100k random boxes and rays (some touching, some degenerate)."""
    import mobileraytracer_amd as m
    rng = np.random.default_rng(3)
    n = 100_000
    lo = rng.normal(size=(n, 3)).astype(F)
    ext = np.abs(rng.normal(size=(n, 3))).astype(F) * (rng.random((n, 3)) > 0.1)  # 10 % flat axes
    boxes = np.concatenate([lo, lo + ext], 1).astype(F)
    orig = (rng.normal(size=(n, 3)) * 3).astype(F)
    orig[::7, 0] = boxes[::7, 0]  # origins on a face
    dirs = rng.normal(size=(n, 3)).astype(F)
    out = m.kat_slab(boxes, orig, dirs)
    finite = out[:, 2] == 1
    assert finite.mean() > 0.99
    assert np.array_equal(out[finite, 0], out[finite, 1])
    sel = np.arange(0, n, 97)
    ref = [oracle_mod.kat_aabb(boxes[k, :3], boxes[k, 3:], orig[k], dirs[k]) for k in sel]
    assert out[sel, 0].tolist() == [int(x) for x in ref]
