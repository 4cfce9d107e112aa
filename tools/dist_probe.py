"""Cost of the multi-GPU frame's pieces on one GPU (run under torch.distributed.run, world 1, nccl):
render into the packed shard buffer, + the RCCL gather, + the unpack into the bitmap."""
import os, sys, time
if os.environ.get("Q8") == "1":
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist
import mobileraytracer_amd as m
from mobileraytracer_amd import scenes

torch.cuda.set_device(0)
use_dist = os.environ.get("NODIST") != "1"
first = os.environ.get("RENDERER_FIRST") == "1"  # renderer (and its HIP streams) before the RCCL init
if use_dist and not first:
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
o, l, c = scenes.conference()
cfg = m.Config(width=1920, height=1080, shader=2, sceneIndex=-1, samplesPixel=4, maxDepth=5, objFilePath=o,
               mtlFilePath=l, camFilePath=c, rankIndex=0, rankCount=int(os.environ.get("RANKS", 1)))
r = m.Renderer(cfg)
if use_dist and first:
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
slots = r.scene_info()["pixelSlotsMax"]
packed = torch.zeros(slots, dtype=torch.int32, device="cuda")
bitmap = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda")
ranks = cfg.rankCount
gathered = torch.zeros((ranks, slots), dtype=torch.int32, device="cuda")  # unpack reads every rank's row
sh = torch.cuda.current_stream().cuda_stream
modes = ("render", "render+gather", "render+gather+unpack", "render", "render+gather+unpack") if use_dist else ("render", "render")
for mode in modes:
    for it in range(13):
        if it == 3:
            torch.cuda.synchronize(); t0 = time.perf_counter()
        r.render_frame_device(0, packed.data_ptr(), sh)
        if "gather" in mode:
            dist.gather(packed, [gathered[0]], dst=0)
        if "unpack" in mode:
            r.unpack_gathered(gathered.data_ptr(), bitmap.data_ptr(), sh)
    torch.cuda.synchronize()
    print(f"{mode}: {(time.perf_counter() - t0) / 10 * 1e3:.3f} ms/frame", flush=True)
r.close()
if use_dist:
    dist.destroy_process_group()
