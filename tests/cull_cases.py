"""Adversarial scenes for the conservative t-cull (tests only).

A grazing ray against a large tilted triangle: Moller-Trumbore's determinant (Triangle.cpp:67-70)
is then dominated by rounding, and the reference accepts a hit at t_c far BEFORE the triangle's
own box entry (t_c = lambda * t_plane with lambda = D / D_c < 1).  A small
triangle placed between t_c and the box entry is found first by a near-first walk; culling the
tilted triangle's box against it drops the reference's answer.  The ray below was found by a
float32 search over grazing rays (tools/cull_search.py) and is checked here against the oracle.
"""
import os

import numpy as np

F = np.float32
# the tilted triangle (integer vertices: exact in every loader)
T2 = ((0, 0, 0), (100, 30, 7), (13, -20, 90))
# the grazing ray: MT gives t_c = 81.1089 while the ray enters T2's box at t = 153.838
ORIG = np.array([-26.89532, -50.145428, 154.96362], F)
DIR = np.array([0.17482877, 0.30672428, -0.93560416], F)
T_C, T_BOX = 81.10892, 153.83807


def _q(x):  # snap to the 1/16 grid (exact decimal text for every float parser)
    return np.round(np.asarray(x, np.float64) * 16.0) / 16.0


def front_triangle(t, size=2.0):
    """A small triangle facing the ray, centred on the ray at parameter ~t."""
    c = ORIG.astype(np.float64) + t * DIR.astype(np.float64)
    d = DIR.astype(np.float64)
    a = np.cross(d, [0.0, 0.0, 1.0])
    a /= np.linalg.norm(a)
    b = np.cross(d, a)
    return [_q(c + size * a), _q(c - size * 0.5 * a + size * b), _q(c - size * 0.5 * a - size * b)]


def write_scene(path, with_front=True, front_t=120.0):
    """OBJ / MTL / CAM of T2, optionally the front triangle, and four far filler triangles (so the
    BVH splits: leaves hold at most 4 primitives, BVH.hpp:239-251)."""
    tris = [list(map(_q, T2))]
    if with_front:
        tris.append(front_triangle(front_t))
        # three small triangles beside the front one (off the ray): the SAH split then puts the
        # front triangle in a leaf of its own group, apart from T2
        c = ORIG.astype(np.float64) + front_t * DIR.astype(np.float64)
        for off in ((-6.0, 0.0, 0.0), (0.0, -6.0, 0.0), (-6.0, -6.0, 0.0)):
            o = _q(c + off)
            tris.append([o, o + [1, 0, 0], o + [0, 1, 0]])
    for k in range(4):
        o = np.array([400.0 + 8 * k, 400.0, 400.0])
        tris.append([o, o + [1, 0, 0], o + [0, 1, 0]])
    os.makedirs(path, exist_ok=True)
    obj, mtl, cam = (os.path.join(path, f"adv.{e}") for e in ("obj", "mtl", "cam"))
    with open(mtl, "w") as f:
        f.write("newmtl grey\nKd 0.5 0.5 0.5\nKs 0 0 0\n")
    with open(obj, "w") as f:
        f.write("mtllib adv.mtl\nusemtl grey\n")
        for tri in tris:
            for v in tri:  # the OBJ loader negates x (OBJLoader.cpp:116-118): write -x
                f.write("v %s %s %s\n" % (repr(-float(v[0])), repr(float(v[1])), repr(float(v[2]))))
        for k in range(len(tris)):
            f.write(f"f {3 * k + 1} {3 * k + 2} {3 * k + 3}\n")
    with open(cam, "w") as f:
        f.write("t perspective\np 0 0 -300\nl 0 0 0\nu 0 1 0\nf 45 45\n")
    return obj, mtl, cam
