"""Streaming mode (tuning key 6) against the level-by-level path: same bitmap and ray counts."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import mobileraytracer_amd as m
from mobileraytracer_amd import scenes


def render(cfg, stream):
    with m.Renderer(cfg) as r:
        r.set_tuning(6, stream)
        bm = np.zeros(cfg.width * cfg.height, np.int32)
        t0 = time.perf_counter()
        r.render_frame(bm)
        dt = time.perf_counter() - t0
        st = r.frame_stats()
        return bm, st["rays"], st["shadowRays"], dt


def main():
    o, l, c = scenes.conference()
    cases = [m.Config(width=64, height=64, shader=1, sceneIndex=0),
             m.Config(width=64, height=64, shader=2, sceneIndex=0, samplesPixel=2),
             m.Config(width=160, height=96, shader=2, sceneIndex=-1, samplesPixel=2, maxDepth=5, objFilePath=o,
                      mtlFilePath=l, camFilePath=c),
             m.Config(width=1920, height=1080, shader=2, sceneIndex=-1, samplesPixel=4, maxDepth=5, objFilePath=o,
                      mtlFilePath=l, camFilePath=c)]
    for cfg in cases:
        a = render(cfg, 0)
        b = render(cfg, 1)
        same = np.array_equal(a[0], b[0]) and a[1] == b[1] and a[2] == b[2]
        print(f"{cfg.width}x{cfg.height} shader {cfg.shader}: identical {same}  rays {a[1]} / {b[1]}  shadows {a[2]} / {b[2]}"
              f"  diff pixels {int((a[0] != b[0]).sum())}", flush=True)


main()
