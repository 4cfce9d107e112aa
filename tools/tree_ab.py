"""A/B of the walk tree (MOBILERT_TREE=0 reference topology, 1 SAH regrouping of the reference
leaves) on the C4 frame: two renderers in one process, interleaved rounds, identical images."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mobileraytracer_amd as m
from mobileraytracer_amd import scenes


def main():
    o, l, c = scenes.conference()
    ranks = int(os.environ.get("RANKS", 1))
    rs = {}
    trees = os.environ.get("TREES", "0,1").split(",")
    for tree in trees:
        os.environ["MOBILERT_TREE"] = tree
        cfg = m.Config(width=1920, height=1080, shader=2, sceneIndex=-1, samplesPixel=4, maxDepth=5,
                       objFilePath=o, mtlFilePath=l, camFilePath=c, rankIndex=0, rankCount=ranks)
        rs[tree] = m.Renderer(cfg)
    n = max(1920 * 1080, rs[trees[0]].scene_info()["pixelSlotsMax"])
    bufs = {k: torch.zeros(n, dtype=torch.int32, device="cuda") for k in rs}
    sh = torch.cuda.current_stream().cuda_stream
    res = {k: [] for k in rs}
    for rnd in range(5):
        for k, r in rs.items():
            bm, pk = (bufs[k].data_ptr(), 0) if ranks == 1 else (0, bufs[k].data_ptr())
            r.render_frame_device(bm, pk, sh)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                r.render_frame_device(bm, pk, sh)
            torch.cuda.synchronize()
            res[k].append((time.perf_counter() - t0) / 5 * 1e3)
    for k in rs:
        print(f"tree {k}: frame {np.median(res[k]):.3f} ms (min {np.min(res[k]):.3f})", flush=True)
    for k in trees[1:]:
        print(f"tree {k} identical image:", torch.equal(bufs[trees[0]], bufs[k]))


main()
