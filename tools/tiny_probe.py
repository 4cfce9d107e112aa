"""Per-launch floor of the trace kernels: tiny frames of a trivial scene (Cornell, a handful of
primitives) and of Conference, with the per-ray maximum of node records (counting pass)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import mobileraytracer_amd as m
from mobileraytracer_amd import scenes


def probe(label, cfg, variant):
    with m.Renderer(cfg) as r:
        r.set_tuning(1, variant)
        d = torch.zeros(cfg.width * cfg.height, dtype=torch.int32, device="cuda")
        sh = torch.cuda.current_stream().cuda_stream
        r.set_profiling(counting=True)
        r.render_frame_device(d.data_ptr(), 0, sh)
        cst = r.frame_stats()
        r.set_profiling(timing=True)
        r.render_frame_device(d.data_ptr(), 0, sh)
        acc = None
        for _ in range(5):
            r.render_frame_device(d.data_ptr(), 0, sh)
            st = r.frame_stats()
            cur = np.array([st["levelTraceMs"], st["levelShadowMs"]])
            acc = cur if acc is None else acc + cur
        acc /= 5
        lv = [f"{st['levelRays'][i]}:{acc[0][i] * 1e3:.0f}us/{acc[1][i] * 1e3:.0f}us" for i in range(8) if st["levelRays"][i]]
        print(f"{label:28s} v{variant}: frame {st['frameMs']:.2f} ms, assists {st['assistedSubtrees']}, max ray {st['maxRayMicros']} us, max node records/ray {cst['maxNodeRecordsPerRay']}, "
              f"nodes/ray {cst['nodeRecords'] / max(1, cst['rays']):.1f}  levels(rays:trace/shadow) {' '.join(lv)}", flush=True)


def main():
    o, l, c = scenes.conference()
    v = int(os.environ.get("VARIANT", 14))
    for w in (16, 64):
        probe(f"cornell {w}x{w} pathtracer", m.Config(width=w, height=w, shader=2, sceneIndex=0, samplesPixel=4, maxDepth=5), v)
        probe(f"conference {w}x{w} pathtracer", m.Config(width=w, height=w, shader=2, sceneIndex=-1, samplesPixel=4, maxDepth=5,
                                                        objFilePath=o, mtlFilePath=l, camFilePath=c), v)


main()
