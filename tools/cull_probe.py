"""Node records / triangle tests per ray of the C4 frame with and without the t-cull (counting pass)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import mobileraytracer_amd as m
from mobileraytracer_amd import scenes

o, l, c = scenes.conference()
cfg = m.Config(width=1920, height=1080, shader=2, sceneIndex=-1, samplesPixel=4, maxDepth=5,
               objFilePath=o, mtlFilePath=l, camFilePath=c)
r = m.Renderer(cfg)
d = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda")
sh = torch.cuda.current_stream().cuda_stream
imgs = []
for cull in (1, 0):
    r.set_tuning(2, cull)
    r.set_profiling(counting=True)
    r.render_frame_device(d.data_ptr(), 0, sh)
    torch.cuda.synchronize()
    st = r.frame_stats()
    imgs.append(d.cpu().numpy().copy())
    w = st["walkedRays"]
    print(f"cull {cull}: closest-hit nodes/ray {st['nodeRecords'] / w:.1f} tris/ray {st['triTests'] / w:.2f}  "
          f"shadow nodes/ray {st['shadowNodeRecords'] / st['shadowRays']:.1f} tris/ray {st['shadowTriTests'] / st['shadowRays']:.2f}  "
          f"rays {st['rays']} shadows {st['shadowRays']}", flush=True)
print("identical images:", np.array_equal(imgs[0], imgs[1]), "differing pixels:", int((imgs[0] != imgs[1]).sum()))
