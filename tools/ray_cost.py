"""Per-frame ray-cost extremes of the C4 frame (counting build): node records and triangle tests
per ray on average and for the costliest single ray, closest hit and shadow."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mobileraytracer_amd as m
from mobileraytracer_amd import scenes


def main():
    o, l, c = scenes.conference()
    ranks = int(os.environ.get("RANKS", 1))
    cfg = m.Config(width=1920, height=1080, shader=2, sceneIndex=-1, samplesPixel=4, maxDepth=5,
                   objFilePath=o, mtlFilePath=l, camFilePath=c, rankIndex=0, rankCount=ranks)
    r = m.Renderer(cfg)
    d = torch.zeros(max(1920 * 1080, r.scene_info()["pixelSlotsMax"]), dtype=torch.int32, device="cuda")
    bm, pk = (d.data_ptr(), 0) if ranks == 1 else (0, d.data_ptr())
    sh = torch.cuda.current_stream().cuda_stream
    for cull in (1, 0, 2):
        r.set_tuning(2, cull)
        r.set_profiling(counting=True)
        r.render_frame_device(bm, pk, sh)
        st = r.frame_stats()
        print(f"cull {cull}: closest {st['nodeRecords'] / max(1, st['walkedRays']):.1f} nodes/ray, "
              f"{st['triTests'] / max(1, st['walkedRays']):.2f} tris/ray; shadow "
              f"{st['shadowNodeRecords'] / max(1, st['shadowRays']):.1f} nodes/ray; max node records of one ray "
              f"{st['maxNodeRecordsPerRay']}", flush=True)


main()
