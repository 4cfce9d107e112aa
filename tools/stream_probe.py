"""Rank 0's C4 shard of an N-GPU frame on one GPU, ms per frame, with or without a process group
(RCCL, world size 1, a collective run so its streams exist) created BEFORE the renderer.

    python tools/stream_probe.py [--pg-first] [--ranks 8] [--frames 20]

Prints one JSON line.  The renderer's shadow walks overlap the next level only while its shadow
stream and the render stream sit on different hardware queues;
tests/test_gpu_parity.py::test_shadow_overlap_survives_rccl_streams compares the two orders."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--pg-first", action="store_true")
    p.add_argument("--ranks", type=int, default=8)
    p.add_argument("--frames", type=int, default=20)
    # normal-priority streams created (and used) before the renderer, as a front end's own streams
    # would be: with HIP's 4 hardware queues per pool they make a later normal-priority stream share
    # a queue with the render stream
    p.add_argument("--extra-streams", type=int, default=0)
    a = p.parse_args()
    import torch
    import torch.distributed as dist
    import mobileraytracer_amd as m
    from mobileraytracer_amd import scenes
    torch.cuda.set_device(0)
    if a.pg_first:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        x = torch.ones(1 << 20, device="cuda")
        dist.all_reduce(x)
        packed0 = torch.zeros(1 << 20, dtype=torch.int32, device="cuda")
        dist.gather(packed0, [torch.empty_like(packed0)], dst=0)
        torch.cuda.synchronize()
    extra = [torch.cuda.Stream() for _ in range(a.extra_streams)]
    for st in extra:
        with torch.cuda.stream(st):
            torch.ones(1024, device="cuda").sum()
    torch.cuda.synchronize()
    o, l, c = scenes.conference()
    cfg = m.Config(width=1920, height=1080, shader=2, sceneIndex=-1, samplesPixel=4, maxDepth=5, objFilePath=o,
                   mtlFilePath=l, camFilePath=c, rankIndex=0, rankCount=a.ranks, device=0)
    r = m.Renderer(cfg)
    packed = torch.zeros(r.scene_info()["pixelSlotsMax"], dtype=torch.int32, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        r.render_frame_device(0, packed.data_ptr(), sh)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.frames):
        r.render_frame_device(0, packed.data_ptr(), sh)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.frames * 1e3
    print(json.dumps({"pg_first": a.pg_first, "extra_streams": a.extra_streams, "ranks": a.ranks, "ms_per_frame": ms,
                      "shadow_stream_concurrent": r.scene_info()["shadowStreamConcurrent"],
                      "shadow_streams_tried": r.scene_info()["shadowStreamsTried"],
                      "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}), flush=True)
    r.close()
    if a.pg_first:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
