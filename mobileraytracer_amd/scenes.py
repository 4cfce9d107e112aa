"""Scene files for the render path.

* ``cornell_water()`` / ``teapot()`` — the OBJ/MTL/CAM fixtures of the reference's own
  instrumentation tests (``app/src/androidTest/resources``), copied as data into
  ``tests/golden``.
* ``conference()`` — the benchmark scene.  ``WavefrontOBJs/conference/conference.obj`` is not
  in the reference snapshot (``.MISSING_LARGE_BLOBS:1``), so unless a real file is supplied
  (``MOBILERT_CONFERENCE_OBJ``) a stand-in is generated: a conference room built from the
  reference's own ``conference.mtl`` materials and ``conference.cam`` camera with exactly the
  triangle and light counts the reference's docker smoke test pins for the real scene
  (331,179 triangles, 2 lights; ``scripts/test/docker/dockerfile.sh:118-119``): a carpeted room,
  a long table with a specular top, sixteen office chairs with specular frames, and a two-
  triangle ceiling light panel.  Coordinates are multiples of 1/16 so every loader parses
  them exactly; the file is deterministic (its SHA-256 is pinned in tests).
"""
import hashlib
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
SCENES = os.path.join(REPO, "scenes")

CONFERENCE_TRIANGLES = 331179   # scripts/test/docker/dockerfile.sh:118
CONFERENCE_LIGHTS = 2           # scripts/test/docker/dockerfile.sh:119


def cornell_water():
    d = os.path.join(GOLDEN, "CornellBox")
    return (os.path.join(d, "CornellBox-Water.obj"), os.path.join(d, "CornellBox-Water.mtl"),
            os.path.join(d, "CornellBox-Water.cam"))


def teapot():
    d = os.path.join(GOLDEN, "teapot")
    return os.path.join(d, "teapot.obj"), os.path.join(d, "teapot.mtl"), os.path.join(d, "teapot.cam")


# ---------------------------------------------------------------------------------------------
# conference stand-in generator

Q = 16.0  # coordinate quantum: 1/16


def _rot_y(p, ang):
    c, s = np.cos(ang), np.sin(ang)
    x, y, z = p[..., 0], p[..., 1], p[..., 2]
    return np.stack([c * x + s * z, y, -s * x + c * z], axis=-1)


def _cube_sphere(n, center, half, q=8.0, ang=0.0):
    """Rounded box (superellipsoid with exponent q) tessellated as a cube-sphere: 6 faces x n x n
    quads, no poles, so no degenerate triangles.  Returns (tris[T,3,3], outward hints[T,3])."""
    t = np.linspace(-1.0, 1.0, n + 1)
    uu, vv = np.meshgrid(t, t, indexing="ij")
    tris, hints = [], []
    for axis in range(3):
        for sgn in (-1.0, 1.0):
            pts = np.zeros((n + 1, n + 1, 3))
            a1, a2 = [a for a in range(3) if a != axis]
            pts[..., axis] = sgn
            pts[..., a1] = uu
            pts[..., a2] = vv
            nrm = (np.abs(pts) ** q).sum(-1) ** (1.0 / q)
            pts = pts / nrm[..., None]
            a = pts[:-1, :-1].reshape(-1, 3)
            b = pts[1:, :-1].reshape(-1, 3)
            c = pts[1:, 1:].reshape(-1, 3)
            d = pts[:-1, 1:].reshape(-1, 3)
            tris.append(np.stack([a, b, c], 1))
            tris.append(np.stack([a, c, d], 1))
    tris = np.concatenate(tris, 0)
    hints = tris.mean(1)  # outward direction in local coordinates
    tris = tris * np.asarray(half)
    tris = _rot_y(tris, ang) + np.asarray(center)
    hints = _rot_y(hints * np.asarray(half), ang)
    return tris, hints


def _grid(corner, e1, e2, n1, n2, inward):
    """Planar quad grid (room surfaces); `inward` is the side the normal must face."""
    corner, e1, e2 = (np.asarray(v, dtype=np.float64) for v in (corner, e1, e2))
    i = np.arange(n1 + 1)[:, None, None] / n1
    j = np.arange(n2 + 1)[None, :, None] / n2
    pts = corner + i * e1 + j * e2
    a = pts[:-1, :-1].reshape(-1, 3)
    b = pts[1:, :-1].reshape(-1, 3)
    c = pts[1:, 1:].reshape(-1, 3)
    d = pts[:-1, 1:].reshape(-1, 3)
    tris = np.concatenate([np.stack([a, b, c], 1), np.stack([a, c, d], 1)], 0)
    hints = np.broadcast_to(np.asarray(inward, dtype=np.float64), (len(tris), 3))
    return tris, hints


def _orient_and_quantize(tris, hints):
    """Quantize to 1/16, drop degenerate triangles, and order the vertices so that the
    reference's flat normal normalize(cross(AC, AB)) (Triangle.cpp:336) faces `hints`."""
    tq = np.round(tris * Q) / Q
    ab = tq[:, 1] - tq[:, 0]
    ac = tq[:, 2] - tq[:, 0]
    cr = np.cross(ac, ab)
    area = np.linalg.norm(cr, axis=1)
    keep = area > 1e-3
    flip = (cr * hints).sum(1) < 0
    out = tq.copy()
    out[flip, 1], out[flip, 2] = tq[flip, 2], tq[flip, 1]
    return out[keep]


def _conference_objects():
    """List of (material, tris) for the stand-in room (world coordinates, y up)."""
    objs = []
    X, Y, Z = 1200.0, 1040.0, 1440.0
    add = lambda mat, th: objs.append((mat, _orient_and_quantize(*th)))
    add("mesh21_SG", _grid((-X, 0, -Z), (2 * X, 0, 0), (0, 0, 2 * Z), 40, 40, (0, 1, 0)))       # carpet
    add("mesh16_SG", _grid((-X, Y, -Z), (2 * X, 0, 0), (0, 0, 2 * Z), 40, 40, (0, -1, 0)))      # ceiling
    add("mesh19_SG", _grid((-X, 0, -Z), (0, Y, 0), (0, 0, 2 * Z), 20, 40, (1, 0, 0)))          # walls
    add("mesh19_SG", _grid((X, 0, -Z), (0, Y, 0), (0, 0, 2 * Z), 20, 40, (-1, 0, 0)))
    add("mesh20_SG", _grid((-X, 0, -Z), (2 * X, 0, 0), (0, Y, 0), 40, 20, (0, 0, 1)))
    add("mesh20_SG", _grid((-X, 0, Z), (2 * X, 0, 0), (0, Y, 0), 40, 20, (0, 0, -1)))
    add("mesh13_SG", _cube_sphere(34, (0, 360, 0), (220, 20, 700), q=10.0))                  # table top (Ks)
    add("mesh6_SG", _cube_sphere(8, (0, 180, -450), (40, 160, 40), q=6.0))                   # table pedestals
    add("mesh6_SG", _cube_sphere(8, (0, 180, 450), (40, 160, 40), q=6.0))
    for side in (-1.0, 1.0):
        for i in range(8):
            z = -630.0 + 180.0 * i
            x = side * 330.0
            ang = 0.0 if side > 0 else np.pi
            lx = lambda dx: x + side * dx  # local "outward" offset along x
            add("mesh11_SG", _cube_sphere(24, (lx(0), 230, z), (110, 22, 110), q=6.0, ang=ang))       # seat
            add("mesh11_SG", _cube_sphere(24, (lx(105), 410, z), (16, 130, 100), q=6.0, ang=ang))     # back
            for dz in (-112.0, 112.0):
                add("mesh12_SG", _cube_sphere(8, (lx(20), 310, z + dz), (70, 10, 12), q=6.0, ang=ang))  # arms (Ks)
            add("mesh13_SG", _cube_sphere(6, (lx(0), 125, z), (16, 85, 16), q=4.0, ang=ang))           # gas lift (Ks)
            for k in range(5):
                a = 2.0 * np.pi * k / 5.0 + 0.3
                cx, cz = lx(0) + 62.0 * np.cos(a), z + 62.0 * np.sin(a)
                add("mesh6_SG", _cube_sphere(4, (cx, 34, cz), (66, 9, 12), q=4.0, ang=-a))          # star leg
                cx2, cz2 = lx(0) + 122.0 * np.cos(a), z + 122.0 * np.sin(a)
                add("mesh22_SG", _cube_sphere(6, (cx2, 17, cz2), (17, 17, 17), q=2.0))              # caster
    return objs


def _light_panel():
    # two triangles, emitting downwards, just below the ceiling
    a, b, c, d = (-300.0, 1030.0, -420.0), (300.0, 1030.0, -420.0), (300.0, 1030.0, 420.0), (-300.0, 1030.0, 420.0)
    tris = np.array([[a, b, c], [a, c, d]], dtype=np.float64)
    return _orient_and_quantize(tris, np.array([[0, -1, 0], [0, -1, 0]], dtype=np.float64))


def _write_obj(path, objs):
    verts = np.concatenate([t.reshape(-1, 3) for _, t in objs], 0)
    vi = np.round(verts * Q).astype(np.int64)
    uniq, inv = np.unique(vi, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    lines = ["# MobileRT MI355X conference stand-in (generated by mobileraytracer_amd/scenes.py)",
             "mtllib conference.mtl"]
    coords = uniq.astype(np.float64) / Q
    coords[:, 0] = -coords[:, 0]  # the loader negates X (OBJLoader.cpp:139-141)
    lines.extend("v %.4f %.4f %.4f" % tuple(v) for v in coords)
    off = 0
    for mat, t in objs:
        lines.append("g " + mat)
        lines.append("usemtl " + mat)
        n = len(t)
        idx = inv[off:off + 3 * n].reshape(n, 3) + 1
        off += 3 * n
        lines.extend("f %d %d %d" % tuple(f) for f in idx)
    with open(path, "w") as f:
        f.write("\n".join(lines))
        f.write("\n")


def generate_conference(path):
    objs = _conference_objects()
    total = sum(len(t) for _, t in objs)
    rem = CONFERENCE_TRIANGLES - total
    if rem < 0:
        raise RuntimeError(f"conference stand-in over budget by {-rem} triangles")
    if rem > 0:
        # whiteboard on the far wall: exactly `rem` triangles (a quad grid, plus one triangle if odd)
        rows = 8
        cols = max(1, (rem // 2) // rows)
        th = _grid((-500, 300, 1430), (1000, 0, 0), (0, 500, 0), cols, rows, (0, 0, -1))
        board = _orient_and_quantize(*th)[: rem]
        while len(board) < rem:  # top-up strip along the board's bottom edge
            extra = _orient_and_quantize(*_grid((-500, 250, 1425), (1000, 0, 0), (0, 40, 0),
                                                 rem - len(board), 1, (0, 0, -1)))
            board = np.concatenate([board, extra[: rem - len(board)]], 0)
        objs.append(("mesh5_SG", board))
    objs.append(("light", _light_panel()))
    n = sum(len(t) for m, t in objs if m != "light")
    assert n == CONFERENCE_TRIANGLES, n
    _write_obj(path, objs)


def file_sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def conference():
    """(obj, mtl, cam) of the benchmark scene; generates the stand-in on first use."""
    d = os.path.join(SCENES, "conference")
    mtl = os.path.join(d, "conference.mtl")
    cam = os.path.join(d, "conference.cam")
    real = os.environ.get("MOBILERT_CONFERENCE_OBJ")
    if real:
        return real, mtl, cam
    obj = os.path.join(d, "conference_standin.obj")
    if not os.path.exists(obj):
        tmp = obj + ".tmp.%d" % os.getpid()
        generate_conference(tmp)
        os.replace(tmp, obj)
    return obj, mtl, cam


def is_standin(obj_path):
    return os.path.basename(obj_path) == "conference_standin.obj"
