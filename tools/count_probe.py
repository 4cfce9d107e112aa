"""Node records / triangle tests per ray of the C4 frame for trace variants (counting pass)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mobileraytracer_amd as m
from mobileraytracer_amd import scenes

o, l, c = scenes.conference()
cfg = m.Config(width=1920, height=1080, shader=2, sceneIndex=-1, samplesPixel=4, maxDepth=5, objFilePath=o,
               mtlFilePath=l, camFilePath=c)
with m.Renderer(cfg) as r:
    d = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    for v in [int(x) for x in os.environ.get("VARIANTS", "14,19").split(",")]:
        r.set_tuning(1, v)
        r.set_profiling(counting=True)
        r.render_frame_device(d.data_ptr(), 0, sh)
        s = r.frame_stats()
        print(f"variant {v}: closest nodes/ray {s['nodeRecords'] / s['rays']:.2f} tris/ray {s['triTests'] / s['rays']:.2f}  "
              f"shadow nodes/ray {s['shadowNodeRecords'] / max(1, s['shadowRays']):.2f} tris/ray {s['shadowTriTests'] / max(1, s['shadowRays']):.2f}", flush=True)
