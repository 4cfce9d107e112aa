"""The Android front end's native session (include/mobilert_android.h) from Python.

The reference's Java / Kotlin classes call these through JNI (mobileraytracer_amd/jni/mrt_jni.cpp
keeps the exported names of app/System_dependent/Android_JNI/JNI_layer.cpp); this module is the
same call sequence for tests and tools:

    read_file(path)                      MainActivity.readFile
    initialize(scene, shader, ...)       MainRenderer.rtInitialize -> primitives, or -1 / -2 / -3
    start_render(wait); render_into_bitmap(pixels, n_threads)
                                         DrawView.rtStartRender; MainRenderer.rtRenderIntoBitmap
    state() / fps() / time_renderer() / sample()
                                         RenderTask.rtGetState / rtGetFps / rtGetTimeRenderer / rtGetSample
    stop_render(wait) / finish_render()  DrawView.rtStopRender / MainRenderer.rtFinishRender
    vertices() / colors() / camera()     MainRenderer.rtInit{Vertices,Colors,Camera}Array
    number_of_lights(), resize(size)     DrawView.rtGetNumberOfLights, MainActivity.rtResize
"""
import ctypes

import numpy as np

from . import _native

IDLE, BUSY, FINISHED, STOPPED = 0, 1, 2, 3  # JNI_layer.hpp:12-13

# The bitmaps render threads still write, kept alive as the locked Android bitmap is: each is
# released by its render thread's done callback, once that thread's last frame has returned.
_live = {}
_token = [0]
_DONE = ctypes.CFUNCTYPE(None, ctypes.c_void_p)


@_DONE
def _release(user):
    _live.pop(int(user or 0), None)


def _lib():
    return _native.lib()


def read_file(path: str, data: bytes = None) -> None:
    if data is None:
        with open(path, "rb") as f:
            data = f.read()
    _lib().mrt_android_read_file(path.encode(), data, len(data))


def initialize(scene: int, shader: int, accelerator: int, width: int, height: int, samples_pixel: int = 1,
               samples_light: int = 1, obj_file_path: str = "") -> int:
    c = _native.MrtAndroidConfig(scene, shader, accelerator, width, height, samples_pixel, samples_light,
                                 obj_file_path.encode())
    return int(_lib().mrt_android_initialize(ctypes.byref(c)))


def render_into_bitmap(pixels: np.ndarray, n_threads: int = 1) -> None:
    assert pixels.dtype == np.int32 and pixels.flags["C_CONTIGUOUS"]
    _token[0] += 1
    _live[_token[0]] = pixels
    _lib().mrt_android_render_into_bitmap_cb(ctypes.c_void_p(pixels.ctypes.data), n_threads,
                                             ctypes.cast(_release, ctypes.c_void_p), ctypes.c_void_p(_token[0]))


def wait_render() -> None:
    """Blocks until no render thread is running (every bitmap handed over is released)."""
    _lib().mrt_android_wait_render()


def bitmaps_in_use() -> int:
    return len(_live)


def start_render(wait: bool = False) -> None:
    _lib().mrt_android_start_render(int(wait))


def stop_render(wait: bool = False) -> None:
    _lib().mrt_android_stop_render(int(wait))


def finish_render() -> None:
    _lib().mrt_android_finish_render()


def state() -> int:
    return int(_lib().mrt_android_state())


def fps() -> float:
    return float(_lib().mrt_android_fps())


def time_renderer() -> int:
    return int(_lib().mrt_android_time_renderer())


def sample() -> int:
    return int(_lib().mrt_android_sample())


def number_of_lights() -> int:
    return int(_lib().mrt_android_number_of_lights())


def resize(size: int) -> int:
    return int(_lib().mrt_android_resize(size))


def _floats(fn):
    n = fn(None)
    out = np.zeros(n, np.float32)
    if n > 0:
        fn(ctypes.c_void_p(out.ctypes.data))
    return out


def vertices() -> np.ndarray:
    return _floats(_lib().mrt_android_vertices)


def colors() -> np.ndarray:
    return _floats(_lib().mrt_android_colors)


def camera() -> np.ndarray:
    return _floats(_lib().mrt_android_camera)


def reset() -> None:
    _lib().mrt_android_reset()
