"""A/B of tuning settings on the C4 frame: one renderer per setting in one process, interleaved
rounds, no per-launch events, images compared.  VARIANTS="6=100,6=75+3=1,W=0" (key=value pairs joined
by '+', settings separated by ','; W / C / O / R / Y set MOBILERT_WALK_TREE / MOBILERT_COLLAPSE / MOBILERT_TREE_OPT /
MOBILERT_TREE_ROT / MOBILERT_RAY_ROT for the upload, P Config.maxPathsPerPass); RANKS=N renders rank 0's shard of an N-GPU frame."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mobileraytracer_amd as m
from mobileraytracer_amd import scenes


def main():
    # SCENE=flat: the flat-geometry stand-in
    o, l, c = scenes.conference() if os.environ.get("SCENE", "conference") == "conference" else scenes.conference_flat()
    ranks = int(os.environ.get("RANKS", 1))
    variants = os.environ.get("VARIANTS", "6=100,6=50").split(",")
    rs = {}
    for v in variants:
        # W=0: MOBILERT_WALK_TREE, C=greedy: MOBILERT_COLLAPSE, O=rounds: MOBILERT_TREE_OPT for this renderer's scene upload
        env = {"W": "MOBILERT_WALK_TREE", "C": "MOBILERT_COLLAPSE", "O": "MOBILERT_TREE_OPT", "R": "MOBILERT_TREE_ROT",
               "Y": "MOBILERT_RAY_ROT"}
        for kv in filter(None, v.split("+")):
            k, val = kv.split("=")
            if k in env:
                os.environ[env[k]] = val
        # P=n: Config.maxPathsPerPass (the frame in passes of at most n paths)
        paths = [int(kv.split("=")[1]) for kv in v.split("+") if kv.startswith("P=")]
        cfg = m.Config(width=1920, height=1080, shader=2, sceneIndex=-1, samplesPixel=4, maxDepth=5,
                       objFilePath=o, mtlFilePath=l, camFilePath=c, rankIndex=0, rankCount=ranks,
                       maxPathsPerPass=paths[0] if paths else 0)
        r = m.Renderer(cfg)
        for kv in filter(None, v.split("+")):
            k, val = kv.split("=")
            if k in env:
                os.environ.pop(env[k])
            elif k != "P":
                r.set_tuning(int(k), int(val))
        rs[v] = r
    n = max(1920 * 1080, rs[variants[0]].scene_info()["pixelSlotsMax"])
    bufs = {k: torch.zeros(n, dtype=torch.int32, device="cuda") for k in rs}
    sh = torch.cuda.current_stream().cuda_stream
    res = {k: [] for k in rs}
    for rnd in range(int(os.environ.get("ROUNDS", 5))):
        for k, r in rs.items():
            bm, pk = (bufs[k].data_ptr(), 0) if ranks == 1 else (0, bufs[k].data_ptr())
            r.render_frame_device(bm, pk, sh)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                r.render_frame_device(bm, pk, sh)
            torch.cuda.synchronize()
            res[k].append((time.perf_counter() - t0) / 5 * 1e3)
    import zlib
    for k in rs:
        crc = zlib.crc32(bufs[k].cpu().numpy().tobytes())
        print(f"setting {k}: frame {np.median(res[k]):.3f} ms (min {np.min(res[k]):.3f}) crc {crc:08x}", flush=True)
    for k in variants[1:]:
        print(f"setting {k} identical image:", torch.equal(bufs[variants[0]], bufs[k]))
    if os.environ.get("COUNT") == "1":  # one counting frame per setting: walk statistics
        for k, r in rs.items():
            bm, pk = (bufs[k].data_ptr(), 0) if ranks == 1 else (0, bufs[k].data_ptr())
            r.set_profiling(counting=True)
            r.render_frame_device(bm, pk, sh)
            torch.cuda.synchronize()
            f = r.frame_stats()
            r.set_profiling()
            sr = max(1, f["shadowRays"])
            print(f"counts {k}: closest records/ray {f['nodeRecords'] / max(1, f['walkedRays']):.2f} "
                  f"tris/ray {f['triTests'] / max(1, f['walkedRays']):.2f} | shadow records/ray "
                  f"{f['shadowNodeRecords'] / sr:.2f} tris/ray {f['shadowTriTests'] / sr:.2f} leaves/ray "
                  f"{f['shadowLeafRecords'] / sr:.2f} occluded {f['shadowOccluded'] / sr:.3f}", flush=True)


main()
