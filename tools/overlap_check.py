"""Do kernels of concurrent pipelines overlap?  Renders rank 0 of an N-way shard with PIPES
pipelines; run under rocprofv3 --kernel-trace and read the trace CSV with --analyse."""
import os, sys, csv, collections
if len(sys.argv) > 2 and sys.argv[1] == "--analyse":
    rows = list(csv.DictReader(open(sys.argv[2])))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-30:], r.get("Queue_Id", r.get("Stream_Id", "?")))
          for r in rows if "k_trace" in r["Kernel_Name"] or "k_shadow" in r["Kernel_Name"] or "k_shade<" in r["Kernel_Name"]]
    ks.sort()
    t0 = ks[-60][0]
    for s, e, n, q in ks[-60:]:
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} q{q} {n}")
    sys.exit(0)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mobileraytracer_amd as m
from mobileraytracer_amd import scenes
o, l, c = scenes.conference()
n = int(os.environ.get("RANKS", 8))
cfg = m.Config(width=1920, height=1080, shader=2, sceneIndex=-1, samplesPixel=4, maxDepth=5, objFilePath=o,
               mtlFilePath=l, camFilePath=c, rankIndex=0, rankCount=n)
with m.Renderer(cfg) as r:
    r.set_tuning(5, int(os.environ.get("PIPES", 2)))
    p = torch.zeros(r.scene_info()["pixelSlotsMax"], dtype=torch.int32, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    for _ in range(5):
        r.render_frame_device(0, p.data_ptr(), sh)
    torch.cuda.synchronize()
