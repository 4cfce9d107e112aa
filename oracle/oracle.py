"""ORACLE — TEST INFRASTRUCTURE ONLY (ctypes wrapper of oracle/build/libmrt_oracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
The library is a CPU restatement of the reference render path (see mrt_oracle.cpp's header
for what pins it and where parity is unpinned).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libmrt_oracle.so")


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


class _Cfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("width", "height", "shader", "sceneIndex", "samplesPixel", "samplesLight", "maxDepth")] + \
               [("obj", ctypes.c_char_p), ("mtl", ctypes.c_char_p), ("cam", ctypes.c_char_p)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        vp, P = ctypes.c_void_p, ctypes.POINTER
        f = ctypes.POINTER(ctypes.c_float)
        L.oracle_create.restype = vp
        L.oracle_create.argtypes = [P(_Cfg)]
        L.oracle_destroy.argtypes = [vp]
        L.oracle_num_tiles.argtypes = [vp]
        L.oracle_render.restype = ctypes.c_uint64
        L.oracle_render.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_render_tiles.restype = ctypes.c_uint64
        L.oracle_render_tiles.argtypes = [vp, vp, ctypes.c_int, vp, ctypes.c_int]
        L.oracle_counts.argtypes = [vp, vp]
        L.oracle_primary_hits.argtypes = [vp, vp, vp, vp]
        L.oracle_triangle_bvh.restype = ctypes.c_int64
        L.oracle_triangle_bvh.argtypes = [vp, vp, vp, vp, vp]
        L.oracle_kat_triangle.argtypes = [f, f, f, f, f, ctypes.c_int, f]
        L.oracle_kat_aabb.argtypes = [f, f, f, f]
        L.oracle_aabb_props.argtypes = [f, f, f, f]
        L.oracle_triangle_aabb.argtypes = [f, f, f, f, f]
        L.oracle_kat_plane.argtypes = [f, f, f, f, f]
        L.oracle_plane_aabb.argtypes = [f, f, f, f]
        L.oracle_kat_camera.argtypes = [ctypes.c_char_p, ctypes.c_float, f]
        L.oracle_halton.restype = ctypes.c_float
        L.oracle_halton.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_table.argtypes = [ctypes.c_uint32, vp]
        L.oracle_path_key.restype = ctypes.c_uint32
        L.oracle_path_key.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_sample_index.restype = ctypes.c_uint32
        L.oracle_sample_index.argtypes = [ctypes.c_uint32] * 3
        L.oracle_incremental_avg.restype = ctypes.c_int32
        L.oracle_incremental_avg.argtypes = [ctypes.c_float] * 3 + [ctypes.c_int32] * 2
        L.oracle_fast_arctan.restype = ctypes.c_float
        L.oracle_fast_arctan.argtypes = [ctypes.c_float]
        L.oracle_selftest_partition.argtypes = [ctypes.c_uint32, ctypes.c_int]
        _lib = L
    return _lib


def fvec(*v):
    a = (ctypes.c_float * len(v))(*[float(x) for x in v])
    return a


class Oracle:
    """CPU reference renderer for one configuration (same meaning as mobileraytracer_amd.Config)."""

    def __init__(self, width, height, shader=1, sceneIndex=0, samplesPixel=1, samplesLight=1, maxDepth=6,
                 obj="", mtl="", cam=""):
        self.width, self.height = width, height
        self._keep = [s.encode() for s in (obj, mtl, cam)]
        c = _Cfg(width, height, shader, sceneIndex, samplesPixel, samplesLight, maxDepth, *self._keep)
        self._h = lib().oracle_create(ctypes.byref(c))
        if not self._h:
            raise RuntimeError("oracle could not load the scene")

    def num_tiles(self):
        return lib().oracle_num_tiles(self._h)

    def render(self, bitmap=None, threads=1, first_tile=0, num_tiles=1 << 30):
        if bitmap is None:
            bitmap = np.zeros(self.width * self.height, np.int32)
        rays = lib().oracle_render(self._h, bitmap.ctypes.data, threads, first_tile, num_tiles)
        return bitmap, int(rays)

    def render_tiles(self, tiles, bitmap=None, threads=1):
        if bitmap is None:
            bitmap = np.zeros(self.width * self.height, np.int32)
        t = np.ascontiguousarray(np.asarray(tiles, np.int32))
        rays = lib().oracle_render_tiles(self._h, bitmap.ctypes.data, threads, t.ctypes.data, len(t))
        return bitmap, int(rays)

    def counts(self):
        out = np.zeros(6, np.int64)
        lib().oracle_counts(self._h, out.ctypes.data)
        return dict(zip(("triangles", "lights", "planes", "spheres", "materials", "triangleNodes"), out.tolist()))

    def primary_hits(self):
        n = self.width * self.height
        k, i, t = np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.float32)
        lib().oracle_primary_hits(self._h, k.ctypes.data, i.ctypes.data, t.ctypes.data)
        return k, i, t

    def triangle_bvh(self):
        n = lib().oracle_triangle_bvh(self._h, None, None, None, None)
        nt = self.counts()["triangles"]
        boxes = np.empty((n, 6), np.float32)
        off, cnt, order = np.empty(n, np.int32), np.empty(n, np.int32), np.empty(nt, np.int32)
        lib().oracle_triangle_bvh(self._h, boxes.ctypes.data, off.ctypes.data, cnt.ctypes.data, order.ctypes.data)
        return boxes, off, cnt, order

    def close(self):
        if getattr(self, "_h", None):
            lib().oracle_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


def kat_triangle(a, b, c, orig, direction, from_self=False):
    t = ctypes.c_float()
    hit = lib().oracle_kat_triangle(fvec(*a), fvec(*b), fvec(*c), fvec(*orig), fvec(*direction), int(from_self),
                                    ctypes.byref(t))
    return bool(hit), t.value


def kat_aabb(mn, mx, orig, direction):
    return bool(lib().oracle_kat_aabb(fvec(*mn), fvec(*mx), fvec(*orig), fvec(*direction)))


def aabb_props(mn, mx):
    c, a = fvec(0, 0, 0), ctypes.c_float()
    lib().oracle_aabb_props(fvec(*mn), fvec(*mx), c, ctypes.byref(a))
    return tuple(c), a.value


def triangle_aabb(a, b, c):
    mn, mx = fvec(0, 0, 0), fvec(0, 0, 0)
    lib().oracle_triangle_aabb(fvec(*a), fvec(*b), fvec(*c), mn, mx)
    return tuple(mn), tuple(mx)


def kat_plane(point, normal, orig, direction):
    t = ctypes.c_float()
    hit = lib().oracle_kat_plane(fvec(*point), fvec(*normal), fvec(*orig), fvec(*direction), ctypes.byref(t))
    return bool(hit), t.value


def plane_aabb(point, normal):
    mn, mx = fvec(0, 0, 0), fvec(0, 0, 0)
    lib().oracle_plane_aabb(fvec(*point), fvec(*normal), mn, mx)
    return tuple(mn), tuple(mx)


def kat_camera(path, ratio):
    out = fvec(*([0] * 14))
    if not lib().oracle_kat_camera(path.encode(), ratio, out):
        raise RuntimeError("camera file not parsed")
    v = list(out)
    return dict(position=v[0:3], direction=v[3:6], up=v[6:9], right=v[9:12], hfov=v[12], vfov=v[13])


def halton(index, base=2):
    return lib().oracle_halton(index, base)


def table(seed):
    out = np.empty(1 << 20, np.float32)
    lib().oracle_table(seed, out.ctypes.data)
    return out


def path_key(pixel, sample):
    return lib().oracle_path_key(pixel, sample)


def sample_index(key, tc, purpose):
    return lib().oracle_sample_index(key, tc, purpose)


def incremental_avg(rgb, avg, n):
    return lib().oracle_incremental_avg(rgb[0], rgb[1], rgb[2], avg, n)


def fast_arctan(v):
    return lib().oracle_fast_arctan(v)


def selftest_partition(seed=1, trials=2000):
    return lib().oracle_selftest_partition(seed, trials)
