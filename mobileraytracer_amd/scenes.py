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


# ---------------------------------------------------------------------------------------------
# a second stand-in with the real Conference's flat character: large flat
# wall / floor / table triangles, long thin slivers, abutting and overlapping coplanar panels - the
# shapes that stress a cull bound and the quantized walk tree's margins at full frame, which the
# rounded furniture of conference() does not

def _box(center, half, ang=0.0, tilt=0.0):
    """Axis-aligned box rotated by `tilt` about x then `ang` about y: 12 triangles, outward hints."""
    c = np.asarray(center, dtype=np.float64)
    h = np.asarray(half, dtype=np.float64)
    sx = np.array([-1.0, 1.0])
    corners = np.array([[x, y, z] for x in sx for y in sx for z in sx]) * h
    ct, st = np.cos(tilt), np.sin(tilt)
    y, z = corners[:, 1].copy(), corners[:, 2].copy()
    corners[:, 1], corners[:, 2] = ct * y - st * z, st * y + ct * z
    corners = _rot_y(corners, ang) + c
    faces = [(0, 1, 3, 2), (4, 6, 7, 5), (0, 4, 5, 1), (2, 3, 7, 6), (0, 2, 6, 4), (1, 5, 7, 3)]
    tris = []
    for a, b, cc, d in faces:
        tris.append([corners[a], corners[b], corners[cc]])
        tris.append([corners[a], corners[cc], corners[d]])
    tris = np.asarray(tris)
    hints = tris.mean(1) - c
    return tris, hints


def _fan(center, rx, rz, y, n, up):
    """Elliptic disk as a fan around its centre: n long thin triangles meeting at one point."""
    a = 2.0 * np.pi * np.arange(n + 1) / n
    ring = np.stack([center[0] + rx * np.cos(a), np.full(n + 1, y), center[1] + rz * np.sin(a)], 1)
    ctr = np.array([center[0], y, center[1]])
    tris = np.stack([np.broadcast_to(ctr, (n, 3)), ring[:-1], ring[1:]], 1)
    return tris, np.broadcast_to(np.array([0.0, up, 0.0]), (n, 3))


def _band(center, rx, rz, y0, y1, n):
    """The rim of an elliptic disk: n tall thin quads (2n triangles), outward."""
    a = 2.0 * np.pi * np.arange(n + 1) / n
    ring = np.stack([center[0] + rx * np.cos(a), np.zeros(n + 1), center[1] + rz * np.sin(a)], 1)
    lo, hi = ring + [0, y0, 0], ring + [0, y1, 0]
    tris = np.concatenate([np.stack([lo[:-1], lo[1:], hi[1:]], 1), np.stack([lo[:-1], hi[1:], hi[:-1]], 1)], 0)
    hints = tris.mean(1) - np.array([center[0], (y0 + y1) / 2, center[1]])
    hints[:, 1] = 0.0
    return tris, hints


def _conference_flat_objects():
    objs = []
    X, Y, Z = 1200.0, 1040.0, 1440.0
    add = lambda mat, th: objs.append((mat, _orient_and_quantize(*th)))  # noqa: E731
    # floor: two abutting coplanar carpets with different subdivisions (T-junctions along x = 0)
    add("mesh21_SG", _grid((-X, 0, -Z), (X, 0, 0), (0, 0, 2 * Z), 40, 60, (0, 1, 0)))
    add("mesh29_SG", _grid((0, 0, -Z), (X, 0, 0), (0, 0, 2 * Z), 37, 53, (0, 1, 0)))
    # ceiling: two large triangles, and a coplanar grid of acoustic tiles overlapping them exactly
    add("mesh16_SG", _grid((-X, Y, -Z), (2 * X, 0, 0), (0, 0, 2 * Z), 1, 1, (0, -1, 0)))
    add("mesh17_SG", _grid((-X, Y, -Z), (2 * X, 0, 0), (0, 0, 2 * Z), 30, 36, (0, -1, 0)))
    # walls: two large triangles each, wainscot strips (tall slivers) coplanar in front of them
    add("mesh19_SG", _grid((-X, 0, -Z), (0, Y, 0), (0, 0, 2 * Z), 1, 1, (1, 0, 0)))
    add("mesh19_SG", _grid((X, 0, -Z), (0, Y, 0), (0, 0, 2 * Z), 1, 1, (-1, 0, 0)))
    add("mesh20_SG", _grid((-X, 0, -Z), (2 * X, 0, 0), (0, Y, 0), 1, 1, (0, 0, 1)))
    add("mesh20_SG", _grid((-X, 0, Z), (2 * X, 0, 0), (0, Y, 0), 1, 1, (0, 0, -1)))
    add("mesh28_SG", _grid((-X, 0, -Z), (0, 300, 0), (0, 0, 2 * Z), 1, 240, (1, 0, 0)))
    add("mesh28_SG", _grid((X, 0, -Z), (0, 300, 0), (0, 0, 2 * Z), 1, 240, (-1, 0, 0)))
    # window blinds on both side walls: tilted slats, thin boxes of long slivers
    for side in (-1.0, 1.0):
        for k in range(60):
            add("mesh9_SG", _box((side * (X - 40), 420 + 8 * k, 0), (2, 0.5, 500), tilt=0.5 * side))
    # table: a fan-triangulated elliptic top (slivers to its centre), its rim, thin legs (mesh13: Ks)
    add("mesh13_SG", _fan((0.0, 0.0), 240.0, 720.0, 380.0, 512, 1.0))
    add("mesh13_SG", _fan((0.0, 0.0), 240.0, 720.0, 372.0, 512, -1.0))
    add("mesh13_SG", _band((0.0, 0.0), 240.0, 720.0, 372.0, 380.0, 512))
    for lx in (-150.0, 150.0):
        for lz in (-600.0, 600.0):
            add("mesh6_SG", _box((lx, 186, lz), (3, 186, 3)))
    # paper sheets stacked on the table: parallel planes 1/16 apart, overlapping in plan
    for k in range(40):
        cx, cz = -160.0 + 80.0 * (k % 5), -600.0 + 150.0 * (k // 5)
        for j in range(25):
            y = 380.0 + (j + 1) / 16.0
            add("mesh5_SG", _grid((cx - 40 + j, y, cz - 55), (80, 0, 0), (0, 0, 110), 1, 1, (0, 1, 0)))
    # chairs: frames of thin bars, slatted seats and backs (mesh11 / mesh12: Ks)
    for side in (-1.0, 1.0):
        for i in range(8):
            z = -630.0 + 180.0 * i
            x = side * 340.0
            for k in range(20):  # seat slats
                add("mesh11_SG", _box((x, 230, z - 95 + 10 * k), (100, 2, 4)))
            for k in range(20):  # back bars
                add("mesh11_SG", _box((x + side * 100, 400, z - 95 + 10 * k), (2, 150, 3)))
            for dx in (-90.0, 90.0):
                for dz in (-90.0, 90.0):
                    add("mesh12_SG", _box((x + dx, 114, z + dz), (2, 114, 2)))  # legs
            for dz in (-100.0, 100.0):
                add("mesh12_SG", _box((x, 300, z + dz), (90, 3, 3)))  # arms
    return objs


def generate_conference_flat(path):
    objs = _conference_flat_objects()
    total = sum(len(t) for _, t in objs)
    rem = CONFERENCE_TRIANGLES - total
    if rem < 0:
        raise RuntimeError(f"flat conference stand-in over budget by {-rem} triangles")
    # the bulk: louvred acoustic panelling on the far wall, 1/2 x 20 slivers (aspect 40), abutting
    # and coplanar, 40 rows; any remainder as one strip of slivers
    Z = 1440.0
    rows = 40
    cols = (rem // 2) // rows
    if cols > 0:
        add_t = _orient_and_quantize(*_grid((-cols / 4.0, 100, Z - 1), (cols / 2.0, 0, 0), (0, 800, 0), cols, rows,
                                            (0, 0, -1)))
        objs.append(("mesh20_SG", add_t))
    rem = CONFERENCE_TRIANGLES - sum(len(t) for _, t in objs)
    if rem > 0:
        strip = _orient_and_quantize(*_grid((-600, 920, Z - 2), (1200, 0, 0), (0, 40, 0), rem, 1, (0, 0, -1)))
        objs.append(("mesh23_SG", strip[:rem]))
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


def conference_flat():
    """(obj, mtl, cam) of the second, flat-geometry Conference stand-in (generate_conference_flat):
    the same camera, materials and pinned counts, built from large flat triangles, slivers and
    coplanar panels."""
    d = os.path.join(SCENES, "conference")
    obj = os.path.join(d, "conference_flat_standin.obj")
    if not os.path.exists(obj):
        tmp = obj + ".tmp.%d" % os.getpid()
        generate_conference_flat(tmp)
        os.replace(tmp, obj)
    return obj, os.path.join(d, "conference.mtl"), os.path.join(d, "conference.cam")


def is_standin(obj_path):
    return os.path.basename(obj_path) in ("conference_standin.obj", "conference_flat_standin.obj")
