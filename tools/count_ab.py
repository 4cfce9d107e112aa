"""Counting-build statistics of the C4 frame per setting (VARIANTS as tools/tune_ab.py): child
records and triangle tests per closest-hit and shadow ray."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mobileraytracer_amd as m
from mobileraytracer_amd import scenes

o, l, c = scenes.conference()
env = {"W": "MOBILERT_WALK_TREE"}
for v in os.environ.get("VARIANTS", "W=0,W=1").split(","):
    kvs = [kv.split("=") for kv in filter(None, v.split("+"))]
    for k, val in kvs:
        if k in env:
            os.environ[env[k]] = val
    cfg = m.Config(width=1920, height=1080, shader=2, sceneIndex=-1, samplesPixel=4, maxDepth=5,
                   objFilePath=o, mtlFilePath=l, camFilePath=c)
    r = m.Renderer(cfg)
    for k, val in kvs:
        if k in env:
            os.environ.pop(env[k])
        else:
            r.set_tuning(int(k), int(val))
    d = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda")
    r.set_profiling(counting=True)
    r.render_frame_device(d.data_ptr(), 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    s = r.frame_stats()
    w, sh = max(1, s["walkedRays"]), max(1, s["shadowRays"])
    print(f"{v}: closest {s['nodeRecords'] / w:.2f} child rec, {s['triTests'] / w:.2f} tris | "
          f"shadow {s['shadowNodeRecords'] / sh:.2f} child rec, {s['shadowTriTests'] / sh:.2f} tris", flush=True)
    r.close() if hasattr(r, "close") else None
