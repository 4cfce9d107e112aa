"""Per-phase lane occupancy of the persistent walks at HEAD: one counting frame of the C4 frame
(and rank 0's shard of the 8-way split), printing, per walk (closest hit at levels >= 2 and the
any-hit shadow walk), the wave iterations of the inner-node phase, the leaf phase and the triangle
loop and the mean active lanes of 64 in them.  The counting build adds the counters only to the
counting instantiation; the timed kernels carry none of them."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mobileraytracer_amd as m
from mobileraytracer_amd import scenes


def run(ranks, scene="conference"):
    o, l, c = scenes.conference() if scene == "conference" else scenes.conference_flat()
    cfg = m.Config(width=1920, height=1080, shader=2, sceneIndex=-1, samplesPixel=4, maxDepth=5,
                   objFilePath=o, mtlFilePath=l, camFilePath=c, rankIndex=0, rankCount=ranks)
    r = m.Renderer(cfg)
    n = max(1920 * 1080, r.scene_info()["pixelSlotsMax"])
    buf = torch.zeros(n, dtype=torch.int32, device="cuda")
    bm, pk = (buf.data_ptr(), 0) if ranks == 1 else (0, buf.data_ptr())
    sh = torch.cuda.current_stream().cuda_stream
    r.render_frame_device(bm, pk, sh)
    r.set_profiling(counting=True)
    r.render_frame_device(bm, pk, sh)
    torch.cuda.synchronize()
    f = r.frame_stats()
    p = list(f["walkPhases"])
    out = {"scene": scene, "ranks": ranks, "walkedRays": f["walkedRays"], "shadowRays": f["shadowRays"]}
    for w, name in enumerate(("closest", "shadow")):
        for k, ph in enumerate(("inner", "leaf", "triangle")):
            it, ln = p[6 * w + 2 * k], p[6 * w + 2 * k + 1]
            out[f"{name}_{ph}_iters"] = it
            out[f"{name}_{ph}_lanes_mean"] = round(ln / max(1, it), 2)
            out[f"{name}_{ph}_occupancy"] = round(ln / max(1, it) / 64, 4)
        it = max(1, p[6 * w])
        out[f"{name}_inner_idle_lanes_mean"] = round(p[12 + 2 * w] / it, 2)   # no ray (waiting for a refill)
        out[f"{name}_inner_done_lanes_mean"] = round(p[13 + 2 * w] / it, 2)   # ray finished, not yet written
    return out


if __name__ == "__main__":
    # usage: phase_occupancy.py [conference|flat] ...   (default: conference)
    for scene in (sys.argv[1:] or ["conference"]):
        for ranks in (1, 8):
            print(json.dumps(run(ranks, scene)), flush=True)
