"""CPU: the quantized 4-wide walk tree by construction.  The GPU walk is
exact because (1) its leaves are exactly the reference BVH's leaves (BVH.hpp:161-283), each once,
and (2) every child box holds the exact box of every reference leaf below it with a margin of at
least one grid step on every side - the margin that covers the rounding of the kernel's
fma(q, step/d, (origin - o)/d) and of the reference's (b - o) * inv.  Both are checked here on the
host build the renderer uploads (mrt_walk_tree), in float64."""
import numpy as np
import pytest

from test_gpu_parity import make_cfg

EMPTY = 0x7FFFFFFE


def _leaf_key(ref):
    v = -ref - 1
    return v >> 3, v & 7


@pytest.mark.parametrize("opt", [None, "0", "100"])
@pytest.mark.parametrize("case", [dict(scene="conference"), dict(scene="water"), dict(scene="teapot"),
                                  dict(sceneIndex=2), dict(sceneIndex=3), dict(scene="conference_flat")])
def test_walk_tree_holds_reference_leaves_with_margin(case, opt, monkeypatch):
    """... for the default build, without the insertion-based optimisation of the tree over the
    leaves (MOBILERT_TREE_OPT=0) and with up to 100 rounds of it."""
    import mobileraytracer_amd as m
    if opt is not None:
        monkeypatch.setenv("MOBILERT_TREE_OPT", opt)
    cfg = make_cfg(64, 64, **case)
    boxes, off, cnt, _ = m.triangle_bvh(cfg)
    leaves = {(int(off[i]), int(cnt[i])): boxes[i].astype(np.float64) for i in range(len(cnt)) if cnt[i] > 0}
    nodes, grid, root = m.walk_tree(cfg)
    width = int(root[2])
    assert width in (4, 8) and nodes.shape[1] == 4 * width
    refs = nodes[:, 3 * width:].view(np.int32)
    org, step = grid[:3].astype(np.float64), grid[3:].astype(np.float64)
    if not leaves:  # no triangles: nothing to walk
        assert int(root[1]) == 0
        return
    assert np.all(step > 0) and int(root[1]) == sum(c for _, c in leaves)
    if int(root[0]) < 0:  # the root is a leaf: no inner node
        assert _leaf_key(int(root[0])) in leaves
        return
    seen = []
    union = {}  # node -> exact union box of the reference leaves below (float64)

    def child_box(ref):
        if ref < 0:
            key = _leaf_key(ref)
            seen.append(key)
            return leaves[key]
        return union[ref]

    # post-order over the 4-wide nodes
    order, stack = [], [int(root[0])]
    while stack:
        i = stack.pop()
        order.append(i)
        stack.extend(int(r) for r in refs[i] if 0 <= int(r) != EMPTY)
    for i in reversed(order):
        w = nodes[i, :3 * width].astype(np.int64)
        u = None
        for c in range(width):
            ref = int(refs[i, c])
            if ref == EMPTY:
                continue
            exact = child_box(ref)
            # one word per axis: min | max << 16
            q = np.array([w[3 * c] & 0xFFFF, w[3 * c + 1] & 0xFFFF, w[3 * c + 2] & 0xFFFF,
                          w[3 * c] >> 16, w[3 * c + 1] >> 16, w[3 * c + 2] >> 16], np.float64)
            qmin, qmax = org + q[:3] * step, org + q[3:] * step
            assert np.all(qmin <= exact[:3] - step), (i, c)
            assert np.all(qmax >= exact[3:] + step), (i, c)
            u = exact.copy() if u is None else np.concatenate([np.minimum(u[:3], exact[:3]), np.maximum(u[3:], exact[3:])])
        union[i] = u
    # every reference leaf exactly once, nothing else
    assert sorted(seen) == sorted(leaves.keys())
    # the root's union is the reference root box
    assert np.array_equal(union[int(root[0])].astype(np.float32), boxes[0])


def _wide_node_area(nodes, grid, width):
    """Summed surface area of the walk tree's wide nodes (each the union of its child boxes, from
    the quantized words): the exact-mode walk's expected visit cost up to a constant."""
    refs = nodes[:, 3 * width:].view(np.int32)
    org, step = grid[:3].astype(np.float64), grid[3:].astype(np.float64)
    w = nodes[:, :3 * width].astype(np.int64).reshape(len(nodes), width, 3)
    lo = org + (w & 0xFFFF) * step
    hi = org + (w >> 16) * step
    used = (refs != EMPTY)[:, :, None]
    lo = np.where(used, lo, np.inf).min(1)
    hi = np.where(used, hi, -np.inf).max(1)
    d = hi - lo
    return float((d[:, 0] * d[:, 1] + d[:, 1] * d[:, 2] + d[:, 2] * d[:, 0]).sum())


@pytest.mark.parametrize("case", [dict(scene="conference"), dict(scene="water"), dict(scene="teapot")])
def test_optimal_collapse_beats_greedy(case, monkeypatch):
    """The wide tree's collapse (mrt_scene.cpp toQuantizedBVH4) minimises the summed area of the
    wide nodes by dynamic programming; the greedy collapse (MOBILERT_COLLAPSE=greedy) is one of
    the trees it considers, so its sum is never larger (up to the quantization's outward step)."""
    import mobileraytracer_amd as m
    cfg = make_cfg(64, 64, **case)
    monkeypatch.setenv("MOBILERT_COLLAPSE", "area")  # (the default weighs nodes by the frame's rays)
    nodes, grid, root = m.walk_tree(cfg)
    monkeypatch.setenv("MOBILERT_COLLAPSE", "greedy")
    gnodes, ggrid, groot = m.walk_tree(cfg)
    width = int(root[2])
    assert int(root[1]) == int(groot[1])
    a_opt, a_greedy = _wide_node_area(nodes, grid, width), _wide_node_area(gnodes, ggrid, width)
    assert a_opt <= a_greedy * 1.0001, (a_opt, a_greedy)
    assert len(nodes) <= len(gnodes)


@pytest.mark.parametrize("case", [dict(scene="conference"), dict(scene="conference_flat"), dict(scene="water"),
                                  dict(scene="teapot")])
def test_tree_optimisation_lowers_the_summed_area(case, monkeypatch):
    """Insertion-based optimisation of the tree over the reference leaves (mrt_scene.cpp
    optimizeOverLeaves) lowers the summed inner-node area of the BVH2 it starts from; after the
    4-wide collapse the wide nodes' summed area (the exact walk's expected visits) must not grow
    beyond the quantization's outward step, and the conference stand-in's falls by >= 3 %."""
    import mobileraytracer_amd as m
    cfg = make_cfg(64, 64, **case)
    monkeypatch.setenv("MOBILERT_COLLAPSE", "area")
    monkeypatch.setenv("MOBILERT_TREE_OPT", "0")
    n0, g0, r0 = m.walk_tree(cfg)
    monkeypatch.setenv("MOBILERT_TREE_OPT", "100")
    n1, g1, r1 = m.walk_tree(cfg)
    width = int(r0[2])
    assert int(r0[1]) == int(r1[1])
    a0, a1 = _wide_node_area(n0, g0, width), _wide_node_area(n1, g1, width)
    assert a1 <= a0 * 1.0001, (a1, a0)
    if case.get("scene") == "conference":
        assert a1 <= a0 * 0.97, (a1, a0)


@pytest.mark.parametrize("case", [dict(scene="conference"), dict(scene="conference_flat"), dict(scene="water"),
                                  dict(scene="teapot")])
def test_wide_rotations_lower_the_wide_area(case, monkeypatch):
    """Rotations of the optimised tree kept where they lower the optimal collapse's summed area
    (mrt_scene.cpp rotateForWide, MOBILERT_TREE_ROT sweeps): never a larger wide area than without
    them, the conference stand-in's lower by >= 0.3 %, and the flat stand-in's tree (the sweep:
    its optimised trees are deeper) untouched.  The process's tree cache keys on the settings."""
    import mobileraytracer_amd as m
    cfg = make_cfg(64, 64, **case)
    monkeypatch.setenv("MOBILERT_COLLAPSE", "area")
    monkeypatch.setenv("MOBILERT_TREE_ROT", "0")
    n0, g0, r0 = m.walk_tree(cfg)
    monkeypatch.delenv("MOBILERT_TREE_ROT")
    n1, g1, r1 = m.walk_tree(cfg)
    width = int(r0[2])
    a0, a1 = _wide_node_area(n0, g0, width), _wide_node_area(n1, g1, width)
    assert a1 <= a0 * 1.0001, (a1, a0)
    if case.get("scene") == "conference":
        assert a1 <= a0 * 0.997, (a1, a0)
    if case.get("scene") == "conference_flat":
        assert np.array_equal(n0, n1)
    # built once per reference tree and settings: the same arrays again, from the cache
    n2, g2, r2 = m.walk_tree(cfg)
    assert np.array_equal(n1, n2) and np.array_equal(g1, g2) and np.array_equal(r1, r2)


@pytest.mark.parametrize("case", [dict(scene="conference"), dict(scene="water"), dict(sceneIndex=3)])
def test_unused_slots_hold_inverted_boxes(case):
    """An unused child slot of the walk tree holds min 65535 / max 0 on every axis
    (mrt_scene.cpp toQuantizedBVH4), which the kernel's near / far slab test (qslabNF) misses
    without a slot check: near > far on the axis for every ray with |qb| <= 4 * 65535 |qa| and a
    normal qa (quantOK), checked here on random such rays with the fma's exact value rounded once."""
    import mobileraytracer_amd as m
    cfg = make_cfg(64, 64, **case)
    nodes, grid, root = m.walk_tree(cfg)
    if int(root[0]) < 0:
        return
    width = int(root[2])
    refs = nodes[:, 3 * width:].view(np.int32)
    words = nodes[:, :3 * width].reshape(len(nodes), width, 3)
    empty = refs == EMPTY
    assert np.all(words[empty] == 0x0000FFFF)
    assert np.all((words[~empty] & 0xFFFF) <= (words[~empty] >> 16))  # used slots: min <= max
    rng = np.random.default_rng(5)
    qa = (rng.choice([-1.0, 1.0], 20000) * 2.0 ** rng.uniform(-100, 60, 20000)).astype(np.float32)
    qb = (qa.astype(np.float64) * rng.uniform(-4 * 65535, 4 * 65535, 20000)).astype(np.float32)
    f32 = lambda x: x.astype(np.float32)  # noqa: E731  (products of a 16-bit q and qa are exact in float64)
    lo = f32(65535.0 * qa.astype(np.float64) + qb.astype(np.float64))  # the min plane's fma
    hi = f32(0.0 * qa.astype(np.float64) + qb.astype(np.float64))      # the max plane's fma
    near = np.where(qa > 0, lo, hi)  # the rotated word: near = min plane for qa > 0, else max
    far = np.where(qa > 0, hi, lo)
    assert np.all(near > far)


@pytest.mark.parametrize("collapse", ["area", "greedy"])
@pytest.mark.parametrize("case", [dict(scene="conference"), dict(scene="water"), dict(sceneIndex=3)])
def test_ray_weighted_collapse_keeps_the_leaves(case, collapse, monkeypatch):
    """The default collapse weighs each BVH2 node by a sample of the frame's own rays
    (mrt_scene.cpp frameRayNodeCosts): the same reference leaves, each once, in a tree of no more
    wide nodes than the greedy collapse's, and (for a scene the camera sees) a different tree from
    the area collapse's - a collapse choice only, which the exactness argument does not depend on."""
    import mobileraytracer_amd as m
    cfg = make_cfg(64, 64, **case)
    nodes, grid, root = m.walk_tree(cfg)
    monkeypatch.setenv("MOBILERT_COLLAPSE", collapse)
    onodes, ogrid, oroot = m.walk_tree(cfg)
    assert int(root[1]) == int(oroot[1]) and np.array_equal(grid, ogrid)
    width = int(root[2])

    def leaves(n, r):
        refs = n[:, 3 * width:].view(np.int32)
        out = [int(x) for x in refs.ravel() if int(x) < 0 and int(x) != EMPTY]
        return sorted(out) if int(r[0]) >= 0 else [int(r[0])]

    assert leaves(nodes, root) == leaves(onodes, oroot)
    if collapse == "greedy":
        assert len(nodes) <= len(onodes)
    if collapse == "area" and case.get("scene") == "conference":
        assert not np.array_equal(nodes, onodes)
