"""Per-depth ray counts and trace times of the C4 frame (default trace variant unless VARIANT)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mobileraytracer_amd as m
from mobileraytracer_amd import scenes


def main():
    o, l, c = scenes.conference()
    w, h = int(os.environ.get("W", 1920)), int(os.environ.get("H", 1080))
    cfg = m.Config(width=w, height=h, shader=2, sceneIndex=-1, samplesPixel=int(os.environ.get("SPP", 4)),
                   maxDepth=5, objFilePath=o, mtlFilePath=l, camFilePath=c,
                   rankIndex=0, rankCount=int(os.environ.get("RANKS", 1)))
    r = m.Renderer(cfg)
    if "VARIANT" in os.environ:
        r.set_tuning(1, int(os.environ["VARIANT"]))
    for kv in filter(None, os.environ.get("TUNE", "").split(",")):  # e.g. TUNE=16=2,5=0
        k, v = kv.split("=")
        r.set_tuning(int(k), int(v))
    d = torch.zeros(max(w * h, r.scene_info()["pixelSlotsMax"]), dtype=torch.int32, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    r.set_profiling(timing=True)
    ranks = int(os.environ.get("RANKS", 1))
    bm, pk = (d.data_ptr(), 0) if ranks == 1 else (0, d.data_ptr())
    r.render_frame_device(bm, pk, sh)
    acc = None
    n = 5
    for _ in range(n):
        r.render_frame_device(bm, pk, sh)
        st = r.frame_stats()
        cur = np.array([st["levelTraceMs"], st["levelShadowMs"]])
        acc = cur if acc is None else acc + cur
    acc /= n
    print(f"variant {r.get_tuning(1)}  frame {st['frameMs']:.2f} ms  trace {st['traceMs']:.2f}  "
          f"shadow {st['shadowMs']:.2f}  shade {st['shadeMs']:.2f}")
    print("depth      rays   trace_ms  Grays/s    shadows  shadow_ms  Grays/s")
    for i in range(16):
        rays, sh_rays = st["levelRays"][i], st["levelShadowRays"][i]
        if rays == 0:
            continue
        tms, sms = acc[0][i], acc[1][i]
        print(f"{i + 1:5d} {rays:10d} {tms:9.3f} {rays / max(tms, 1e-9) / 1e6:8.2f} {sh_rays:10d} {sms:9.3f} "
              f"{sh_rays / max(sms, 1e-9) / 1e6:8.2f}")


main()
