"""MI355X-native render hot path of MobileRT (TiagoMSSantos/MobileRayTracer).

Python mirror of the reference's native surface for this path:

* ``Config``            — ``MobileRT::Config`` (app/MobileRT/Config.hpp:12-83)
* ``Renderer``          — ``MobileRT::Renderer`` (app/MobileRT/Renderer.hpp:41-63) as built by
                          ``work_thread`` (app/System_dependent/Native/C_wrapper.cpp:36-211):
                          the constructor assembles scene + shader + BVH + camera, then
                          ``render_frame`` / ``stop_render`` / ``get_sample`` /
                          ``get_total_casted_rays`` keep the reference's meaning.
* ``ray_trace``         — ``RayTrace(Config&, bool)`` (C_wrapper.cpp:268-290).

Everything computes in the HIP kernels of ``libmobilert_amd.so``; there is no CPU path.
"""
import ctypes
import dataclasses
import threading
import time
from typing import List, Optional

import numpy as np

from . import _native

SHADER_WHITTED = 1      # C_wrapper.cpp:155
SHADER_PATH_TRACER = 2  # C_wrapper.cpp:162
ACC_BVH = 3             # Shader.hpp:20-24
RAY_DEPTH_MAX = 6       # Constants.hpp:45


@dataclasses.dataclass
class Config:
    """MobileRT::Config plus the GPU-only knobs of mrt_config."""
    width: int = 256
    height: int = 256
    threads: int = 1
    shader: int = SHADER_WHITTED
    sceneIndex: int = 0
    samplesPixel: int = 1
    samplesLight: int = 1
    repeats: int = 1
    accelerator: int = ACC_BVH
    printStdOut: bool = False
    objFilePath: str = ""
    mtlFilePath: str = ""
    camFilePath: str = ""
    bitmap: Optional[np.ndarray] = None
    maxDepth: int = RAY_DEPTH_MAX
    rankIndex: int = 0
    rankCount: int = 1
    device: int = -1
    cull: int = 3
    maxPathsPerPass: int = 0
    progressive: int = 0
    # a device group: one screen-tile shard per listed HIP device, assembled on devices[0]
    # (mrt_config.devices; empty or one entry: a single GPU, `device`)
    devices: List[int] = dataclasses.field(default_factory=list)

    def to_c(self):
        c = _native.MrtConfig()
        for f in ("width", "height", "threads", "shader", "sceneIndex", "samplesPixel", "samplesLight",
                  "repeats", "accelerator", "maxDepth", "rankIndex", "rankCount", "device", "cull",
                  "maxPathsPerPass", "progressive"):
            setattr(c, f, int(getattr(self, f)))
        c.printStdOut = int(bool(self.printStdOut))
        self._keep = [s.encode() for s in (self.objFilePath, self.mtlFilePath, self.camFilePath)]
        c.objFilePath, c.mtlFilePath, c.camFilePath = self._keep
        if len(self.devices) > 1:
            self._keep_devices = (ctypes.c_int32 * len(self.devices))(*[int(d) for d in self.devices])
            c.devices = self._keep_devices
            c.deviceCount = len(self.devices)
        return c


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


class Renderer:
    def __init__(self, config: Config):
        self._lib = _native.lib()
        self.config = config
        handle = ctypes.c_void_p()
        _native.check(self._lib.mrt_create(ctypes.byref(config.to_c()), ctypes.byref(handle)))
        self._h = handle

    # -- reference Renderer surface ------------------------------------------------------
    def render_frame(self, bitmap: np.ndarray, num_threads: int = 1) -> None:
        """Renderer::renderFrame(int32_t *bitmap, int32_t numThreads); numThreads is unused."""
        del num_threads
        assert bitmap.dtype == np.int32 and bitmap.size == self.config.width * self.config.height
        assert bitmap.flags["C_CONTIGUOUS"]
        _native.check(self._lib.mrt_render_frame(self._h, _ptr(bitmap)))

    def render_frame_device(self, d_bitmap: int = 0, d_packed: int = 0, stream: int = 0) -> None:
        """Frame into device memory (pointers as ints, e.g. torch ``data_ptr()``)."""
        _native.check(self._lib.mrt_render_frame_device(
            self._h, ctypes.c_void_p(d_bitmap or None), ctypes.c_void_p(d_packed or None),
            ctypes.c_void_p(stream or None)))

    def unpack_gathered(self, d_gathered: int, d_bitmap: int, stream: int = 0) -> None:
        _native.check(self._lib.mrt_unpack_gathered(self._h, ctypes.c_void_p(d_gathered),
                                                     ctypes.c_void_p(d_bitmap), ctypes.c_void_p(stream or None)))

    def stop_render(self) -> None:
        _native.check(self._lib.mrt_stop_render(self._h))

    def get_sample(self) -> int:
        return int(self._lib.mrt_get_sample(self._h))

    def get_total_casted_rays(self) -> int:
        return int(self._lib.mrt_get_total_casted_rays(self._h))

    # -- extras --------------------------------------------------------------------------
    def scene_info(self) -> dict:
        info = _native.MrtSceneInfo()
        _native.check(self._lib.mrt_get_scene_info(self._h, ctypes.byref(info)))
        return {f: getattr(info, f) for f, _ in info._fields_}

    def set_profiling(self, timing: bool = False, counting: bool = False) -> None:
        _native.check(self._lib.mrt_set_profiling(self._h, int(timing) | (2 * int(counting))))

    def set_tuning(self, key: int, value: int) -> None:
        """A/B knobs: 1 = trace walk (0 reference, 1 default), 2 = t-cull mode (0 none, 1 fast -
        inexact on grazing inputs, 2 certified, 3 exact: the default), 3 = shadow rays on their own
        stream, 5 = shadow-walk child order (0 near first, 1 far first),
        6 = shadow-walk grid percent (0 auto), 7 = no walk for the depth-capped last level, 8 = tail
        donation (idle lanes of a level's tail walk subtrees of their wave's rays), 9 = refill
        threshold of the walk waves, 10 = lean k_shade instantiation, 11 = k_shade workgroups per CU,
        16 = the camera rays' packet walk (cull modes 0 and 3; refused when the walk tree needs a
        deeper stack than the packet walk's), 17 = level 1 fused (camera rays generated,
        packet-walked and shaded in one launch), 19-23 = the tile kernel and its knobs, 27 = the
        last shadow walk on the render stream.  Results are identical for every value, except
        key 2 = 1 (documented inexact)."""
        _native.check(self._lib.mrt_set_tuning(self._h, key, value))

    def set_camera(self, kind: int, position, look_at, up, a: float, b: float) -> None:
        """mrt_set_camera: kind 0 Perspective(position, lookAt, up, hFov, vFov in degrees), 1
        Orthographic(position, lookAt, up, sizeH, sizeV) (Perspective.cpp / Orthographic.cpp)."""
        vec = lambda v: (ctypes.c_float * 3)(*[float(x) for x in v])  # noqa: E731
        _native.check(self._lib.mrt_set_camera(self._h, kind, vec(position), vec(look_at), vec(up), a, b))

    def set_pixel_sampler(self, kind: int, value: float = 0.5) -> None:
        """mrt_set_pixel_sampler: 0 Constant(value), 1 StaticHaltonSeq (the Renderer's pixel sampler)."""
        _native.check(self._lib.mrt_set_pixel_sampler(self._h, kind, value))

    def set_max_point(self, max_point) -> None:
        """mrt_set_max_point: DepthMap's maxPoint."""
        _native.check(self._lib.mrt_set_max_point(self._h, (ctypes.c_float * 3)(*[float(x) for x in max_point])))

    def get_tuning(self, key: int) -> int:
        v = ctypes.c_int32(0)
        _native.check(self._lib.mrt_get_tuning(self._h, key, ctypes.byref(v)))
        return v.value

    def wave_log(self):
        """Counting mode: the last frame's per-wave log, uint64 [2 (closest, any-hit), 16 levels,
        8192 waves, 4 (start, end in 100 MHz ticks, rays fetched, child records fetched)]."""
        n = int(self._lib.mrt_wave_log(self._h, None))
        out = np.zeros(n, np.uint64)
        _native.check(0 if self._lib.mrt_wave_log(self._h, out.ctypes.data_as(ctypes.c_void_p)) >= 0 else -1)
        return out.reshape(2, 16, 8192, 4)

    def frame_stats(self) -> dict:
        s = _native.MrtFrameStats()
        _native.check(self._lib.mrt_get_frame_stats(self._h, ctypes.byref(s)))
        out = {f: getattr(s, f) for f, _ in s._fields_}
        out["levelRays"] = list(s.levelRays)
        out["levelShadowRays"] = list(s.levelShadowRays)
        out["levelTraceMs"] = list(s.levelTraceMs)
        out["levelShadowMs"] = list(s.levelShadowMs)
        for k in ("levelNodeRecords", "levelTriTests", "levelLeafRecords", "levelShadedVertices", "walkPhases",
                  "packetWaveRecords"):
            out[k] = list(getattr(s, k))
        return out

    def frame_rays(self):
        """(walkedRays, shadowRays) of the last frame: frame_stats()'s two ray counts without building
        its dict (a per-frame call in bench.py's timed loop)."""
        s = getattr(self, "_rays_buf", None)
        if s is None:
            s = self._rays_buf = _native.MrtFrameStats()
        _native.check(self._lib.mrt_get_frame_stats(self._h, ctypes.byref(s)))
        return s.walkedRays, s.shadowRays

    def primary_hits(self):
        """(kind, index, t) per pixel, index in the scene's input order (config C2)."""
        n = self.config.width * self.config.height
        kind = np.empty(n, np.int32)
        index = np.empty(n, np.int32)
        t = np.empty(n, np.float32)
        _native.check(self._lib.mrt_primary_hits(self._h, _ptr(kind), _ptr(index), _ptr(t)))
        return kind, index, t

    def trace_rays(self, orig, dirs, dist=None, src=None, any_hit=False):
        """Arbitrary rays through the trace kernels (current walk / cull): closest hit
        (kind, input index, t) per ray, or with any_hit the shadow test within dist
        (kind = occluded).  src: None or (n, 2) int32 (kind, input index) source primitives."""
        o = np.ascontiguousarray(orig, np.float32)
        d = np.ascontiguousarray(dirs, np.float32)
        n = len(o)
        ds = np.ascontiguousarray(dist if dist is not None else np.zeros(n), np.float32)
        sp = None if src is None else np.ascontiguousarray(src, np.int32)
        k, i, t = np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.float32)
        _native.check(self._lib.mrt_trace_rays(self._h, _ptr(o), _ptr(d), _ptr(ds), None if sp is None else _ptr(sp),
                                               n, int(any_hit), _ptr(k), _ptr(i), _ptr(t)))
        return k, i, t

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.mrt_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def walk_tree(config: Config):
    """Host-side quantized wide walk tree of the configured scene (no GPU): nodes (N, 4W) uint32
    (3W box words, W child references), grid (6,) float32 (origin xyz, step xyz), root (3,) int32
    (reference, triangle count, width W) - DESIGN.md section 3.1."""
    lib = _native.lib()
    c = config.to_c()
    n = lib.mrt_walk_tree(ctypes.byref(c), None, None, None)
    if n < 0:
        raise RuntimeError(lib.mrt_last_error().decode())
    # the width first (a node is 4 * width words), then the nodes
    grid = np.empty(6, np.float32)
    root = np.empty(3, np.int32)
    lib.mrt_walk_tree(ctypes.byref(c), None, _ptr(grid), _ptr(root))
    nodes = np.empty((n, 4 * int(root[2])), np.uint32)
    if lib.mrt_walk_tree(ctypes.byref(c), _ptr(nodes), _ptr(grid), _ptr(root)) != n:
        raise RuntimeError(lib.mrt_last_error().decode())
    return nodes, grid, root


def triangle_bvh(config: Config):
    """Host-side triangle BVH of the configured scene (no GPU): boxes (N, 6), offsets, counts,
    order - the layout of the reference's BVHNode array (BVH.hpp:56-60)."""
    lib = _native.lib()
    c = config.to_c()
    n = lib.mrt_triangle_bvh(ctypes.byref(c), None, None, None, None)
    if n < 0:
        raise RuntimeError(lib.mrt_last_error().decode())
    boxes = np.empty((n, 6), np.float32)
    off, cnt = np.empty(n, np.int32), np.empty(n, np.int32)
    order = np.full((n + 1) // 2, -1, np.int32)  # 2 * triangles - 1 slots (a lone root: 0 or 1 triangle)
    n2 = lib.mrt_triangle_bvh(ctypes.byref(c), _ptr(boxes), _ptr(off), _ptr(cnt), _ptr(order))
    if n2 != n:
        raise RuntimeError(lib.mrt_last_error().decode())
    return boxes, off, cnt, order[:int(cnt[0])] if n == 1 else order


def regular_grid(config: Config, kind: int):
    """Host-side RegularGrid (accelerator 2, RegularGrid.hpp with gridSize 32) of one primitive
    kind of the configured scene (0 planes, 1 spheres, 2 triangles), no GPU: world (12 floats:
    min, max, cellSize, cellSizeInverted), start (32^3 + 1), items (input indices)."""
    lib = _native.lib()
    c = config.to_c()
    n = lib.mrt_regular_grid(ctypes.byref(c), kind, None, None, None)
    if n < 0:
        raise RuntimeError(lib.mrt_last_error().decode())
    world, start, items = np.empty(12, np.float32), np.empty(32 ** 3 + 1, np.int32), np.empty(max(n, 1), np.int32)
    if lib.mrt_regular_grid(ctypes.byref(c), kind, _ptr(world), _ptr(start), _ptr(items)) != n:
        raise RuntimeError(lib.mrt_last_error().decode())
    return world, start, items[:n]


def grid_box_test(kind: int, prim, box) -> bool:
    """The RegularGrid fill's cell membership test (Triangle / Plane / Sphere::intersect(const
    AABB&)) as the renderer's host build evaluates it.  kind 0 prim = A + B + C, 1 = point +
    normal, 2 = center + (radius,); box = min + max."""
    p = np.ascontiguousarray(prim, np.float32)
    b = np.ascontiguousarray(box, np.float32)
    rc = _native.lib().mrt_grid_box_test(kind, _ptr(p), _ptr(b))
    if rc < 0:
        raise ValueError(_native.lib().mrt_last_error().decode())
    return bool(rc)


def decode_texture(path: str) -> np.ndarray:
    """A map_Kd texture decoded as the renderer loads it (Texture::createTexture,
    Texture.cpp:83-114): (height, width, channels) uint8.  Host only."""
    lib = _native.lib()
    dims = np.zeros(3, np.int32)
    n = lib.mrt_decode_texture(path.encode(), _ptr(dims), None)
    if n < 0:
        raise RuntimeError(lib.mrt_last_error().decode())
    out = np.empty(int(n), np.uint8)
    lib.mrt_decode_texture(path.encode(), _ptr(dims), _ptr(out))
    return out.reshape(int(dims[1]), int(dims[0]), int(dims[2]))


def sample_tables():
    """Host only: (shader table, sampler table, trig (2^20 x cos, sin)) as the renderer builds them."""
    a, b, t = np.empty(1 << 20, np.float32), np.empty(1 << 20, np.float32), np.empty(2 << 20, np.float32)
    _native.check(_native.lib().mrt_sample_tables(_ptr(a), _ptr(b), _ptr(t)))
    return a, b, t.reshape(-1, 2)


def kat_slab(boxes, orig, dirs):
    """The device slab test (AABB.cpp:34-54) on (box, ray) pairs: (reference predicate,
    IEEE-min/max form, 1/d finite) per pair, int32 (n, 3)."""
    b = np.ascontiguousarray(boxes, np.float32)
    o = np.ascontiguousarray(orig, np.float32)
    d = np.ascontiguousarray(dirs, np.float32)
    out = np.empty((len(b), 3), np.int32)
    _native.check(_native.lib().mrt_kat_slab(_ptr(b), _ptr(o), _ptr(d), len(b), _ptr(out)))
    return out


def kat_triangle(tris, orig, dirs):
    """The device triangle test (Triangle.cpp:63-109) on (triangle A B C, ray) pairs: hit, t."""
    tr = np.ascontiguousarray(tris, np.float32)
    o = np.ascontiguousarray(orig, np.float32)
    d = np.ascontiguousarray(dirs, np.float32)
    hit, t = np.empty(len(tr), np.int32), np.empty(len(tr), np.float32)
    _native.check(_native.lib().mrt_kat_triangle(_ptr(tr), _ptr(o), _ptr(d), len(tr), _ptr(hit), _ptr(t)))
    return hit, t


_active: List[Renderer] = []


def ray_trace(config: Config, async_: bool = False):
    """RayTrace(Config&, bool) (C_wrapper.cpp:36-290): build, render `repeats` frames into
    config.bitmap, print the reference's summary lines."""
    def work():
        if config.bitmap is None:
            config.bitmap = np.zeros(config.width * config.height, np.int32)
        t0 = time.perf_counter()
        # progressive, as C_wrapper's render loop: the caller may read config.bitmap meanwhile
        r = Renderer(dataclasses.replace(config, progressive=1))
        t1 = time.perf_counter()
        _active.append(r)
        try:
            repeats = config.repeats
            t2 = time.perf_counter()
            while True:
                r.render_frame(config.bitmap, config.threads)
                repeats -= 1
                if repeats <= 0:
                    break
            secs = time.perf_counter() - t2
            rays = r.get_total_casted_rays()
            if config.printStdOut:
                info = r.scene_info()
                print(f"TRIANGLES = {info['triangles']}")
                print(f"LIGHTS = {info['lights']}")
                print(f"Creating Time in secs = {t1 - t0}")
                print(f"Rendering Time in secs = {secs}")
                print(f"Casted rays = {rays}")
                print(f"width = {config.width}")
                print(f"height = {config.height}")
                print(f"Total Millions rays per second = {rays / secs / 1e6}")
        finally:
            _active.remove(r)
            r.close()
    if async_:
        th = threading.Thread(target=work, daemon=True)
        th.start()
        return th
    work()
    return None


def stop_render():
    """stopRender() (C_wrapper.cpp:271-275)."""
    for r in list(_active):
        r.stop_render()
