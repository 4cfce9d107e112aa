"""Benchmark: Mrays/s and ms/frame of the MobileRT render path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json metric, configs[3] = C4): the Conference scene at 1920x1080,
4 samples per pixel, PathTracer, RayDepthMax 5 (camera ray + 4 bounces), samplesLight 1.
A step is one Renderer::renderFrame (all 4 samples).  "Rays" counts every ray constructed
(camera, shadow, diffuse, specular, transmission), as the reference's Ray id counter does
(Ray.cpp:25-28; C_wrapper.cpp:247-256).  The frame buffer stays in device memory; the
reference's host-bitmap copy is excluded (DESIGN.md gives the PCIe-inclusive rate).

Multi-GPU: one process per GPU; the frame's screen tiles are sharded (unit u -> rank u % N),
each rank renders its shard into a packed buffer, one RCCL gather brings the shards to rank 0,
which scatters them into the bitmap.  Total work is one frame whatever N is: scaling "strong".
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

BASELINE_METRIC = "Mrays/s + ms/frame, Conference OBJ 1920\u00d71080 4spp, 1/2/4/8 GPU"  # BASELINE.json "metric"
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
PEAK_L2_GBS = 34500.0  # aggregate L2 (8 x 4 MiB) read rate, same guide, section "L2 (per XCD)"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--spp", type=int, default=4)
    p.add_argument("--max-depth", type=int, default=5)
    p.add_argument("--shader", type=int, default=2)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-tiles", type=int, default=64, help="tiles of the frame timed on the CPU oracle")
    return p.parse_args()


def cpu_baseline(args, scene):
    """The oracle (CPU restatement, AoS + recursion + std::thread tiles) on a bounded sample of
    the same workload: every 4th reference tile (64 of 256) of the same frame."""
    from oracle import oracle as O
    threads = min(16, os.cpu_count() or 1)
    o = O.Oracle(args.width, args.height, args.shader, -1, args.spp, 1, args.max_depth,
                 obj=scene[0], mtl=scene[1], cam=scene[2])
    tiles = list(range(0, o.num_tiles(), max(1, o.num_tiles() // args.cpu_tiles)))[: args.cpu_tiles]
    t0 = time.perf_counter()
    _, rays = o.render_tiles(tiles, threads=threads)
    dt = time.perf_counter() - t0
    o.close()
    return {"value": rays / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{len(tiles)} of 256 reference tiles (every 4th) of the same frame, {rays} rays, {dt:.1f} s"}


def pmc_traffic_per_launch():
    """HBM bytes per k_trace launch from the committed rocprofv3 PMC summary, if present."""
    path = os.path.join(HERE, "profiles", "pmc_trace_kernel.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get("hbm_bytes_per_launch")


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import mobileraytracer_amd as m
    from mobileraytracer_amd import scenes

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MRT_BENCH_BACKEND=gloo (rehearsal only: several ranks sharing one GPU, gather through host
    # memory); the measured multi-GPU path is RCCL ("nccl") with one GPU per rank
    backend = os.environ.get("MRT_BENCH_BACKEND", "nccl")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        local = local % torch.cuda.device_count() if backend == "gloo" else local
        torch.cuda.set_device(local)
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    scene = scenes.conference()
    cfg = m.Config(width=args.width, height=args.height, shader=args.shader, sceneIndex=-1,
                   samplesPixel=args.spp, samplesLight=1, maxDepth=args.max_depth, objFilePath=scene[0],
                   mtlFilePath=scene[1], camFilePath=scene[2], rankIndex=rank, rankCount=world,
                   device=torch.cuda.current_device())
    r = m.Renderer(cfg)
    info = r.scene_info()
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    slots_max = info["pixelSlotsMax"]
    bitmap = torch.zeros(args.width * args.height, dtype=torch.int32, device="cuda")
    packed = torch.zeros(slots_max, dtype=torch.int32, device="cuda")
    gathered = torch.zeros((world, slots_max), dtype=torch.int32, device="cuda") if rank == 0 else None

    def step():
        if world == 1:
            r.render_frame_device(bitmap.data_ptr(), 0, sh)
        else:
            r.render_frame_device(0, packed.data_ptr(), sh)
            if backend == "gloo":
                host = packed.cpu()
                parts = [torch.empty_like(host) for _ in range(world)] if rank == 0 else None
                dist.gather(host, parts, dst=0)
                if rank == 0:
                    gathered.copy_(torch.stack(parts))
            else:
                dist.gather(packed, list(gathered.unbind(0)) if rank == 0 else None, dst=0)
            if rank == 0:
                r.unpack_gathered(gathered.data_ptr(), bitmap.data_ptr(), sh)

    for _ in range(args.warmup):
        step()
    # one counting frame (outside the timed region): node / triangle fetches per ray
    trace_variant = r.get_tuning(1)
    r.set_profiling(counting=True)
    step()
    counted = r.frame_stats()
    r.set_profiling(timing=True)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    rays0 = r.get_total_casted_rays()
    t0 = time.perf_counter()
    trace_ms = 0.0
    trace_launches = 0
    walked = 0  # closest-hit rays traversed + shadow rays: the rays whose walk ran
    for _ in range(args.steps):
        step()
        st = r.frame_stats()
        trace_ms += st["traceMs"]
        trace_launches += st["traceLaunches"]
        walked += st["walkedRays"] + st["shadowRays"]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    rays = r.get_total_casted_rays() - rays0

    if world > 1:
        red = "cpu" if backend == "gloo" else "cuda"
        t = torch.tensor([elapsed], dtype=torch.float64, device=red)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        n = torch.tensor([rays, walked], dtype=torch.float64, device=red)
        dist.all_reduce(n, op=dist.ReduceOp.SUM)
        rays, walked = [int(x) for x in n.tolist()]
        agg = torch.tensor([counted["walkedRays"], counted["nodeRecords"], counted["triTests"], trace_ms,
                            trace_launches], dtype=torch.float64, device=red)
        dist.all_reduce(agg, op=dist.ReduceOp.SUM)
        c_rays, c_nodes, c_tris, trace_ms, trace_launches = [float(x) for x in agg.tolist()]
    else:
        c_rays, c_nodes, c_tris = counted["walkedRays"], counted["nodeRecords"], counted["triTests"]

    if rank != 0:
        dist.destroy_process_group()
        return

    # roofline of the dominant kernel (k_trace, closest hit), SURVEY.md section 8(d):
    # B_ray = 32 (ray read) + 16 (hit write) + 32 * N_node + 36 * N_tri, summed over the
    # frame's closest-hit rays; per launch = frame bytes / launches per frame
    frames = max(1, args.steps)
    launches_per_frame = trace_launches / frames
    bytes_per_frame = 48.0 * c_rays + 32.0 * c_nodes + 36.0 * c_tris
    bytes_per_launch = bytes_per_frame / max(1.0, launches_per_frame)  # launches of all ranks
    avg_launch_ms = trace_ms / max(1.0, trace_launches)
    achieved = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9 if avg_launch_ms > 0 else 0.0
    traffic = pmc_traffic_per_launch() if world == 1 else None
    out = {
        "metric": BASELINE_METRIC,
        # rays whose walk ran: the depth-capped last level's rays (built, shaded to zero, walk
        # skipped) are not counted; rays_built_per_frame is the reference's ray count
        "value": walked / elapsed / 1e6,
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / frames * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic" if scenes.is_standin(scene[0]) else "conference.obj",
        "config": {
            "workload": f"conference_{args.width}x{args.height}_{args.spp}spp_pathtracer_depth{args.max_depth}",
            "scene": ("conference stand-in: 331179 triangles + 2 area lights, reference conference.mtl/.cam "
                      "(conference.obj is absent from the reference snapshot)") if scenes.is_standin(scene[0])
            else scene[0],
            "resolution": [args.width, args.height],
            "rendered_pixels": int(info["pixelSlots"]) if world == 1 else None,
            "spp": args.spp, "max_depth": args.max_depth, "samples_light": 1,
            "shader": "PathTracer" if args.shader == 2 else "Whitted",
            "parallelism": (f"screen-tile shard x{world} + " + ("RCCL gather" if backend == "nccl" else "gloo gather (rehearsal)"))
            if world > 1 else "single GPU",
            "rays_walked_per_frame": walked / frames,
            "rays_built_per_frame": rays / frames,
            "mrays_per_s_built": rays / elapsed / 1e6,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_trace (closest hit)",
            "achieved": achieved,
            "peak": PEAK_HBM_GBS,
            "unit": "GB/s",
            "frac": achieved / PEAK_HBM_GBS,
            "traffic": traffic,
            "avg_launch_ms": avg_launch_ms,
            "algorithmic_bytes_per_launch": bytes_per_launch,
            "per_ray": {"nodes": c_nodes / max(1.0, c_rays), "tris": c_tris / max(1.0, c_rays)},
            "frac_of_l2_peak": achieved / PEAK_L2_GBS,
            "note": ("node/triangle gathers hit in L2 and the 256 MiB Infinity Cache (the Conference "
                     "working set is ~30 MB), so algorithmic bytes/s is not capped by HBM; `traffic` "
                     "is the rocprofv3-measured bytes beyond L2 per launch (profiles/pmc_trace_kernel.json)"),
            "trace_variant": trace_variant,
        },
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, scene)
    print(json.dumps(out), flush=True)
    r.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
