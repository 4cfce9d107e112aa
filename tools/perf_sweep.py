"""A/B the trace-kernel variants on the C4 frame in one process (interleaved rounds)."""
import os, sys, json, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mobileraytracer_amd as m
from mobileraytracer_amd import scenes

def main():
    o, l, c = scenes.conference()
    # RANKS=N: rank 0's shard of an N-GPU frame (packed output), the per-GPU work at N GPUs
    ranks = int(os.environ.get("RANKS", 1))
    cfg = m.Config(width=1920, height=1080, shader=2, sceneIndex=-1, samplesPixel=4, maxDepth=5,
                   objFilePath=o, mtlFilePath=l, camFilePath=c, rankIndex=0, rankCount=ranks)
    r = m.Renderer(cfg)
    d = torch.zeros(max(1920 * 1080, r.scene_info()["pixelSlotsMax"]), dtype=torch.int32, device="cuda")
    bm, pk = (d.data_ptr(), 0) if ranks == 1 else (0, d.data_ptr())
    sh = torch.cuda.current_stream().cuda_stream
    # "V[:O[:K[:C[:B]]]]": trace walk V (0 reference, 1 default), shadow-stream overlap O (default 1),
    # last-level walk skip K (default 1), t-cull C (default 1), binned emission B (default 0),
    # shadow-walk child order A (0 near first, default 1 far first): "V:O:K:C:B:A"
    variants = os.environ.get("VARIANTS", "1,1:0").split(",")
    imgs = {}
    res = {v: [] for v in variants}
    r.set_profiling(timing=True)
    for rnd in range(3):
        for v in variants:
            parts = v.split(":")
            parts += ["1", "1", "1", "0", "1"][len(parts) - 1:]
            r.set_tuning(1, int(parts[0]))
            r.set_tuning(3, int(parts[1]))
            r.set_tuning(7, int(parts[2]))  # skip the last level's walk (default 1)
            r.set_tuning(2, int(parts[3]))  # near-first + t-cull (default 1)
            r.set_tuning(4, int(parts[4]))  # binned emission (default 0)
            r.set_tuning(5, int(parts[5]))  # shadow walk child order (default 1: far first)
            r.render_frame_device(bm, pk, sh)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = 5
            tr = shw = shd = 0.0
            for _ in range(n):
                r.render_frame_device(bm, pk, sh)
                st = r.frame_stats()
                tr += st["traceMs"]; shw += st["shadowMs"]; shd += st["shadeMs"]
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / n
            rays = st["rays"] + st["shadowRays"]
            res[v].append((dt * 1e3, tr / n, shw / n, rays / dt / 1e6, shd / n))
            imgs[v] = d.cpu().numpy().copy()
    for v in variants:
        a = np.array(res[v])
        print(f"variant {v}: frame {np.median(a[:,0]):.2f} ms  trace {np.median(a[:,1]):.2f}  shadow {np.median(a[:,2]):.2f}  shade {np.median(a[:,4]):.2f}  Mrays/s {np.median(a[:,3]):.0f}", flush=True)
    base = imgs[variants[0]]
    for v in variants[1:]:
        print(f"variant {v} identical image: {np.array_equal(base, imgs[v])}")

main()
