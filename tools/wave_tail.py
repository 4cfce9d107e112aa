"""Wave-level timeline of the walk launches of one C4 frame (counting build, RANKS=N shard):
per level, when the waves of k_trace / k_shadow end relative to the launch's first start, and
how many rays the last waves fetched.  Shows whether a level's time is its bulk or its tail."""
import os, sys
import numpy as np
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
    for kv in filter(None, os.environ.get("TUNE", "").split("+")):
        k, v = kv.split("=")
        r.set_tuning(int(k), int(v))
    d = torch.zeros(max(1920 * 1080, r.scene_info()["pixelSlotsMax"]), dtype=torch.int32, device="cuda")
    bm, pk = (d.data_ptr(), 0) if ranks == 1 else (0, d.data_ptr())
    sh = torch.cuda.current_stream().cuda_stream
    r.set_profiling(counting=True)
    r.render_frame_device(bm, pk, sh)
    r.render_frame_device(bm, pk, sh)
    torch.cuda.synchronize()
    log = r.wave_log().astype(np.int64)
    for kind, name in ((0, "trace"), (1, "shadow")):
        for lev in range(1, 16):
            e = log[kind, lev]
            ran = e[:, 1] > 0
            if not ran.any():
                continue
            e = e[ran]
            t0 = e[:, 0].min()
            end = (e[:, 1] - t0) / 100.0  # us
            start = (e[:, 0] - t0) / 100.0
            q = np.percentile(end, [10, 50, 90, 99, 100])
            late = end > np.percentile(end, 99)
            print(f"{name} L{lev}: waves {ran.sum()} rays {e[:, 2].sum()} start max {start.max():.1f} us | end p10 {q[0]:.0f} "
                  f"p50 {q[1]:.0f} p90 {q[2]:.0f} p99 {q[3]:.0f} max {q[4]:.0f} us | rays/wave mean {e[:, 2].mean():.0f}, "
                  f"late 1%: {e[late, 2].mean():.0f} rays {e[late, 3].mean() / max(1, e[late, 2].mean()):.0f} rec/ray "
                  f"(all {e[:, 3].sum() / max(1, e[:, 2].sum()):.0f})", flush=True)


main()
