"""ctypes binding of libmobilert_amd.so (include/mobilert_amd.h).

This is the stub a Python front end (or the test-suite) uses in place of the reference's
native bindings; INTEGRATION.md shows the JNI / Qt equivalents.  The library is built
in-tree by ``__graft_entry__.build()`` (``make -C mobileraytracer_amd/csrc``).  There is no
CPU fallback: if the shared object is missing, importing this module raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MOBILERT_LIB: another build of the library (A/B of compile-time variants, tools/build_ab.sh)
LIB_PATH = os.environ.get("MOBILERT_LIB") or os.path.join(_HERE, "libmobilert_amd.so")

# Symbols the C-ABI exports (include/mobilert_amd.h + mobilert_amd.hpp).
EXPORTED_SYMBOLS = (
    "mrt_last_error", "mrt_build_stamp", "mrt_create", "mrt_destroy", "mrt_render_frame", "mrt_render_frame_device",
    "mrt_unpack_gathered", "mrt_stop_render", "mrt_get_sample", "mrt_get_total_casted_rays",
    "mrt_get_scene_info", "mrt_set_profiling", "mrt_get_frame_stats", "mrt_primary_hits", "mrt_set_tuning",
    "mrt_get_tuning", "mrt_triangle_bvh", "mrt_walk_tree", "mrt_decode_texture", "mrt_kat_slab", "mrt_kat_triangle",
    "mrt_trace_rays", "mrt_sample_tables", "mrt_regular_grid", "mrt_grid_box_test", "mrt_create_from_memory",
    "mrt_preview_arrays", "mrt_wave_log", "mrt_set_camera", "mrt_set_pixel_sampler", "mrt_set_max_point",
    "mrt_android_read_file", "mrt_android_initialize", "mrt_android_render_into_bitmap",
    "mrt_android_render_into_bitmap_cb", "mrt_android_wait_render", "mrt_android_start_render",
    "mrt_android_stop_render", "mrt_android_finish_render", "mrt_android_state", "mrt_android_fps",
    "mrt_android_time_renderer", "mrt_android_sample", "mrt_android_number_of_lights", "mrt_android_resize",
    "mrt_android_vertices", "mrt_android_colors", "mrt_android_camera", "mrt_android_reset",
    "RayTrace", "stopRender",
)


class MrtConfig(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32), ("height", ctypes.c_int32), ("threads", ctypes.c_int32),
        ("shader", ctypes.c_int32), ("sceneIndex", ctypes.c_int32), ("samplesPixel", ctypes.c_int32),
        ("samplesLight", ctypes.c_int32), ("repeats", ctypes.c_int32), ("accelerator", ctypes.c_int32),
        ("printStdOut", ctypes.c_int32),
        ("objFilePath", ctypes.c_char_p), ("mtlFilePath", ctypes.c_char_p), ("camFilePath", ctypes.c_char_p),
        ("maxDepth", ctypes.c_int32), ("rankIndex", ctypes.c_int32), ("rankCount", ctypes.c_int32),
        ("device", ctypes.c_int32), ("cull", ctypes.c_int32), ("maxPathsPerPass", ctypes.c_int32),
        ("progressive", ctypes.c_int32), ("devices", ctypes.POINTER(ctypes.c_int32)), ("deviceCount", ctypes.c_int32),
    ]


class MrtAndroidConfig(ctypes.Structure):  # include/mobilert_android.h
    _fields_ = [(n, ctypes.c_int32) for n in (
        "scene", "shader", "accelerator", "width", "height", "samplesPixel", "samplesLight")] + [
        ("objFilePath", ctypes.c_char_p)]


class MrtBlob(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("bytes", ctypes.c_char_p), ("size", ctypes.c_int64)]


class MrtSceneInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in (
        "triangles", "lights", "planes", "spheres", "materials", "triangleNodes", "triangleBvhDepth",
        "pixelSlots", "pixelSlotsMax", "deviceBytes", "shadowStreamConcurrent", "shadowStreamsTried", "deviceCount")]


class MrtFrameStats(ctypes.Structure):
    _fields_ = [
        ("rays", ctypes.c_uint64), ("shadowRays", ctypes.c_uint64), ("primaryRays", ctypes.c_uint64),
        ("nodeRecords", ctypes.c_uint64), ("triTests", ctypes.c_uint64),
        ("shadowNodeRecords", ctypes.c_uint64), ("shadowTriTests", ctypes.c_uint64),
        ("traceMs", ctypes.c_double), ("shadowMs", ctypes.c_double), ("frameMs", ctypes.c_double),
        ("traceLaunches", ctypes.c_int64), ("shadowLaunches", ctypes.c_int64),
        ("shadeMs", ctypes.c_double),
        ("levelRays", ctypes.c_uint64 * 16), ("levelShadowRays", ctypes.c_uint64 * 16),
        ("levelTraceMs", ctypes.c_double * 16), ("levelShadowMs", ctypes.c_double * 16),
        ("maxNodeRecordsPerRay", ctypes.c_uint64),
        ("walkedRays", ctypes.c_uint64), ("shadedVertices", ctypes.c_uint64), ("shadeLaunches", ctypes.c_int64),
        ("leafRecords", ctypes.c_uint64), ("shadowLeafRecords", ctypes.c_uint64),
        ("levelNodeRecords", ctypes.c_uint64 * 16), ("levelTriTests", ctypes.c_uint64 * 16),
        ("levelLeafRecords", ctypes.c_uint64 * 16),
        ("fusedMs", ctypes.c_double), ("fusedLaunches", ctypes.c_int64),
        ("levelShadedVertices", ctypes.c_uint64 * 16),
        ("shadowOccluded", ctypes.c_uint64),
        ("walkPhases", ctypes.c_uint64 * 16),
        ("packetWaveRecords", ctypes.c_uint64 * 3),
    ]


def _preload_torch_hip_runtime():
    """One HIP runtime per process: if PyTorch-ROCm is installed, load its libamdhip64 first
    (by full path, without importing torch) so this library and torch share it whichever is
    imported first.  Both carry the SONAME libamdhip64.so.7."""
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return
    rt = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(rt):
        ctypes.CDLL(rt, mode=ctypes.RTLD_GLOBAL)


def load_library(path=LIB_PATH):
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the MI355X path has no CPU fallback)")
    _preload_torch_hip_runtime()
    lib = ctypes.CDLL(path)
    P = ctypes.POINTER
    vp = ctypes.c_void_p
    sig = {
        "mrt_last_error": (ctypes.c_char_p, []),
        "mrt_build_stamp": (ctypes.c_char_p, []),
        "mrt_create": (ctypes.c_int, [P(MrtConfig), P(vp)]),
        "mrt_destroy": (None, [vp]),
        "mrt_render_frame": (ctypes.c_int, [vp, vp]),
        "mrt_render_frame_device": (ctypes.c_int, [vp, vp, vp, vp]),
        "mrt_unpack_gathered": (ctypes.c_int, [vp, vp, vp, vp]),
        "mrt_stop_render": (ctypes.c_int, [vp]),
        "mrt_get_sample": (ctypes.c_int32, [vp]),
        "mrt_get_total_casted_rays": (ctypes.c_uint64, [vp]),
        "mrt_get_scene_info": (ctypes.c_int, [vp, P(MrtSceneInfo)]),
        "mrt_set_profiling": (ctypes.c_int, [vp, ctypes.c_int32]),
        "mrt_get_frame_stats": (ctypes.c_int, [vp, P(MrtFrameStats)]),
        "mrt_wave_log": (ctypes.c_int64, [vp, vp]),
        "mrt_primary_hits": (ctypes.c_int, [vp, vp, vp, vp]),
        "mrt_set_tuning": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32]),
        "mrt_get_tuning": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]),
        "mrt_triangle_bvh": (ctypes.c_int64, [vp, vp, vp, vp, vp]),
        "mrt_walk_tree": (ctypes.c_int64, [vp, vp, vp, vp]),
        "mrt_decode_texture": (ctypes.c_int64, [ctypes.c_char_p, vp, vp]),
        "mrt_regular_grid": (ctypes.c_int64, [vp, ctypes.c_int32, vp, vp, vp]),
        "mrt_grid_box_test": (ctypes.c_int, [ctypes.c_int32, vp, vp]),
        "mrt_create_from_memory": (ctypes.c_int, [P(MrtConfig), ctypes.c_char_p, ctypes.c_int64, ctypes.c_char_p,
                                                  ctypes.c_int64, ctypes.c_char_p, ctypes.c_int64, vp, ctypes.c_int32,
                                                  P(vp)]),
        "mrt_preview_arrays": (ctypes.c_int64, [vp, vp, vp, vp]),
        "mrt_set_camera": (ctypes.c_int, [vp, ctypes.c_int32, vp, vp, vp, ctypes.c_float, ctypes.c_float]),
        "mrt_set_pixel_sampler": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_float]),
        "mrt_set_max_point": (ctypes.c_int, [vp, vp]),
        "mrt_android_read_file": (None, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int64]),
        "mrt_android_initialize": (ctypes.c_int32, [P(MrtAndroidConfig)]),
        "mrt_android_render_into_bitmap": (None, [vp, ctypes.c_int32]),
        "mrt_android_render_into_bitmap_cb": (None, [vp, ctypes.c_int32, vp, vp]),
        "mrt_android_wait_render": (None, []),
        "mrt_android_start_render": (None, [ctypes.c_int32]),
        "mrt_android_stop_render": (None, [ctypes.c_int32]),
        "mrt_android_finish_render": (None, []),
        "mrt_android_state": (ctypes.c_int32, []),
        "mrt_android_fps": (ctypes.c_float, []),
        "mrt_android_time_renderer": (ctypes.c_int64, []),
        "mrt_android_sample": (ctypes.c_int32, []),
        "mrt_android_number_of_lights": (ctypes.c_int32, []),
        "mrt_android_resize": (ctypes.c_int32, [ctypes.c_int32]),
        "mrt_android_vertices": (ctypes.c_int64, [vp]),
        "mrt_android_colors": (ctypes.c_int64, [vp]),
        "mrt_android_camera": (ctypes.c_int64, [vp]),
        "mrt_android_reset": (None, []),
        "mrt_sample_tables": (ctypes.c_int, [vp, vp, vp]),
        "mrt_kat_slab": (ctypes.c_int, [vp, vp, vp, ctypes.c_int32, vp]),
        "mrt_kat_triangle": (ctypes.c_int, [vp, vp, vp, ctypes.c_int32, vp, vp]),
        "mrt_trace_rays": (ctypes.c_int, [vp, vp, vp, vp, vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("MOBILERT_LIB") and not hasattr(lib, name):
            continue  # an older A/B build without a newer test entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = load_library()
    return _LIB


def source_stamp():
    """The digest the Makefile embeds (mrt_build_stamp) for the csrc sources in this tree."""
    import hashlib
    d = os.path.join(_HERE, "csrc")
    srcs = ["mrt_scene.cpp", "mrt_grid.cpp", "mrt_texture.cpp", "mrt_android.cpp", "mrt_kernels.hip", "mrt_renderer.hip",
            "mrt_common.hpp", "mrt_device.hpp", "mrt_kernels.hpp", "mrt_trace_ww.hpp", "mrt_trace_packet.hpp",
            "mrt_scene.hpp", "../../include/mobilert_amd.h", "../../include/mobilert_amd.hpp",
            "../../include/mobilert_android.h"]
    h = hashlib.sha256()
    for f in srcs:
        with open(os.path.join(d, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_is_current(library=None):
    """True when the loaded library was built from this tree's sources (no extra flags)."""
    return (library or lib()).mrt_build_stamp().decode() == source_stamp()


def check(rc):
    if rc != 0:
        raise RuntimeError(lib().mrt_last_error().decode(errors="replace"))
