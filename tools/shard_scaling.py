"""Per-rank frame time of one screen-tile shard (rank 0 of N) on one GPU: the work each GPU
does in an N-GPU run, without the gather.  Estimates strong-scaling efficiency T1 / (N * TN)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mobileraytracer_amd as m
from mobileraytracer_amd import scenes


def frame_ms(n, w=1920, h=1080, spp=4, frames=10, rank=0):
    o, l, c = scenes.conference()
    cfg = m.Config(width=w, height=h, shader=2, sceneIndex=-1, samplesPixel=spp, maxDepth=5, objFilePath=o,
                   mtlFilePath=l, camFilePath=c, rankIndex=rank, rankCount=n)
    with m.Renderer(cfg) as r:
        if "OVERLAP" in os.environ:
            r.set_tuning(3, int(os.environ["OVERLAP"]))
        if "VARIANT" in os.environ:
            r.set_tuning(1, int(os.environ["VARIANT"]))
        packed = torch.zeros(r.scene_info()["pixelSlotsMax"], dtype=torch.int32, device="cuda")
        sh = torch.cuda.current_stream().cuda_stream
        for _ in range(3):
            r.render_frame_device(0, packed.data_ptr(), sh)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(frames):
            r.render_frame_device(0, packed.data_ptr(), sh)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / frames * 1e3


def main():
    if "ALLRANKS" in os.environ:
        n = int(os.environ["ALLRANKS"])
        ts = [frame_ms(n, rank=k, frames=5) for k in range(n)]
        t1 = frame_ms(1, frames=5)
        print(f"N={n} per-rank ms: " + " ".join(f"{t:.2f}" for t in ts) + f"  max {max(ts):.2f}  efficiency {t1 / (n * max(ts)):.3f}")
        return
    w, h, spp = int(os.environ.get("W", 1920)), int(os.environ.get("H", 1080)), int(os.environ.get("SPP", 4))
    t1 = None
    for n in (1, 2, 4, 8):
        t = frame_ms(n, w, h, spp)
        t1 = t if t1 is None else t1
        print(f"{w}x{h} spp {spp}  N={n}: rank-0 shard {t:.2f} ms/frame, efficiency {t1 / (n * t):.3f}", flush=True)


main()
