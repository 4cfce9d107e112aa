"""Benchmark: Mrays/s and ms/frame of the MobileRT render path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Both forms run N ranks, one process per GPU.  Without a launcher (WORLD_SIZE unset) and N > 1,
this process starts the N rank processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT set, before anything touches the GPU), forwards their output (rank 0 prints the
line) and exits with the worst of their return codes.  It refuses, non-zero and before any GPU
call, N larger than the visible GPUs (RCCL: one GPU per rank) and, under a launcher, N != WORLD_SIZE.

Workload (BASELINE.json metric, configs[3] = C4): the Conference scene at 1920x1080,
4 samples per pixel, PathTracer, RayDepthMax 5 (camera ray + 4 bounces), samplesLight 1.
A step is one Renderer::renderFrame (all 4 samples).  `value` is WALKED Mrays/s: every ray
whose BVH walk ran (camera, diffuse, specular and shadow rays; the depth-capped last level's
rays are built and counted by the reference but shade to zero without a walk, DESIGN.md
section 3).  The reference's own count, every Ray constructed (Ray.cpp:25-28,
C_wrapper.cpp:247-256), is `config.mrays_per_s_built`.  The frame buffer stays in device
memory; the reference's host-bitmap copy is excluded (DESIGN.md gives the PCIe-inclusive rate).
The timed frames run with per-launch event timing OFF.

Per-kernel roofline: outside the timed region one counting frame (node / triangle fetches per
ray, shaded vertices) and two frames with the shadow stream serialised and HIP events around
every launch give each kernel's average launch duration; `achieved` = algorithmic bytes per
launch / that duration.

Multi-GPU: one process per GPU; the frame's pixel units (reference tile t cut into 8-row bands b)
are sharded unit (t, b) -> rank (t + b) % N; each rank renders its shard into a packed buffer,
one RCCL gather brings the shards to rank 0, which scatters them into the bitmap.  Total work
is one frame whatever N is: scaling "strong".  `--path group` times the same partition the way
the front ends run it (RayTrace / the C++ facade / the Android session with MOBILERT_DEVICES):
one process, one Renderer over a device group, one long-lived shard worker thread per GPU, the
shards assembled on the first GPU by peer copies.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

BASELINE_METRIC = "Mrays/s + ms/frame, Conference OBJ 1920×1080 4spp, 1/2/4/8 GPU"  # BASELINE.json "metric"
# /opt/skills/guides/MI355X_MICROARCH.md: HBM 8.0 TB/s peak; L2 34.5 TB/s aggregate, 36.9 TB/s
# with the L1-reuse contribution: the most the vector-memory path delivers to the CUs, the
# ceiling of a gather-bound kernel whose working set is cache-resident
PEAK_HBM_GBS = 8000.0
PEAK_VMEM_GBS = 36900.0


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
    p.add_argument("--overlap", type=int, default=1, help="shadow rays on their own stream (timed frames)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    # rehearsals (not the headline line): rank 0's shard of an N-GPU frame on this one GPU (e.g.
    # C5: --width 3840 --height 2160 --spp 8 --shard-of 8), and the final bitmap saved as .npy
    p.add_argument("--shard-of", type=int, default=0)
    p.add_argument("--dump-bitmap", default="")
    # the scene: the Conference stand-in (default) or the flat-geometry stand-in (rehearsal lines)
    p.add_argument("--scene", choices=("conference", "flat"), default="conference")
    # the multi-GPU form: "ranks" (default) one process per GPU over RCCL; "group" one process and
    # one Renderer over a device group (mrt_config.devices: the front ends' own multi-GPU path,
    # RayTrace / the C++ facade / the Android session with MOBILERT_DEVICES), shards assembled by
    # peer copies.  The group's ordinals: MOBILERT_DEVICES if set (e.g. "0,0,0,0" rehearses four
    # shards on one GPU), else 0 .. N-1.
    p.add_argument("--path", choices=("ranks", "group"), default="ranks")
    return p.parse_args()


def group_devices(gpus, env):
    """The device ordinals of `--path group`: MOBILERT_DEVICES (the front ends' variable, parsed as
    the library does: whole non-negative decimal ordinals) or 0 .. gpus-1."""
    s = env.get("MOBILERT_DEVICES", "")
    if not s:
        return list(range(gpus))
    out = []
    for item in s.split(","):
        if not item.isdigit():
            raise ValueError(f"MOBILERT_DEVICES: bad ordinal '{item}'")
        out.append(int(item))
    return out


def launch_plan(gpus, env, device_count, path="ranks"):
    """What `bench.py --gpus N` does in this process: ("run", None) renders here (one rank, or one
    rank of a launcher's world, or the whole device group of `--path group`); ("spawn", N) starts N
    rank processes; ("error", message).  Decided from the environment and the device count alone
    (torch.cuda.device_count() does not initialise the GPU), so the parent of spawned ranks never
    touches the GPU."""
    if gpus < 1:
        return "error", f"--gpus must be >= 1 (got {gpus})"
    if path == "group":
        if "WORLD_SIZE" in env and int(env["WORLD_SIZE"]) != 1:
            return "error", "--path group renders the whole frame from one process: run it without a launcher"
        try:
            devs = group_devices(gpus, env)
        except ValueError as e:
            return "error", str(e)
        if len(devs) != gpus:
            return "error", f"--gpus {gpus} but MOBILERT_DEVICES lists {len(devs)} device(s)"
        bad = [d for d in devs if d >= device_count]
        if bad:
            return "error", f"device group ordinal {bad[0]} but {device_count} visible GPU(s)"
        return "run", None
    backend = env.get("MRT_BENCH_BACKEND", "nccl")
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            return "error", f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks"
        local_world = int(env.get("LOCAL_WORLD_SIZE", world))
        if backend == "nccl" and local_world > device_count:
            return "error", (f"{local_world} ranks on this node but {device_count} visible GPU(s): "
                             "RCCL needs one GPU per rank")
        return "run", None
    if gpus > 1 and backend == "nccl" and gpus > device_count:
        return "error", f"--gpus {gpus} but {device_count} visible GPU(s): RCCL needs one GPU per rank"
    return ("spawn", gpus) if gpus > 1 else ("run", None)


def spawn_ranks(n, argv):
    """Start n rank processes of this script (one per GPU; the torch.distributed.run environment)
    and wait for them.  A rank that fails ends the others (their own PIDs); returns the worst code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for rank in range(n):
        env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    worst = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0:
                worst = worst or rc
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    for p in procs:
        rc = p.wait()
        if rc != 0 and worst == 0:
            worst = rc
    return worst


def effective_cores():
    """Host threads this process may use: its CPU affinity, capped by a cgroup CPU quota."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, scene):
    """The oracle (CPU restatement of the reference: AoS triangles, by-value hit records, the
    reference's DFS, recursive shaders, std::thread tile loop) in timing-faithful mode (the
    reference's shared atomic sampler cursors) over the WHOLE frame, on every core this
    process may use."""
    from oracle import oracle as O
    threads = effective_cores()
    o = O.Oracle(args.width, args.height, args.shader, -1, args.spp, 1, args.max_depth,
                 obj=scene[0], mtl=scene[1], cam=scene[2])
    o.set_faithful(True)
    load_before = os.getloadavg() if hasattr(os, "getloadavg") else None
    c0 = time.process_time()
    t0 = time.perf_counter()
    _, rays = o.render(threads=threads)
    dt = time.perf_counter() - t0
    cpu_s = time.process_time() - c0
    load_after = os.getloadavg() if hasattr(os, "getloadavg") else None
    o.close()
    return {"value": rays / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            # the box's load explains the baseline's box-to-box swing: the per-core rate is the rays over
            # the CPU seconds this process got, and utilisation is how many of `cores` it actually ran on
            "per_core_value": rays / cpu_s / 1e6 if cpu_s > 0 else None,
            "utilisation": cpu_s / dt / threads if dt > 0 else None,
            "loadavg_1_5_15_before": load_before, "loadavg_1_5_15_after": load_after,
            "host_cpus_visible": os.cpu_count(),
            "cpu_model": cpu_model(),
            "sample": f"full frame (all 256 reference tiles, {args.spp} spp), {rays} rays built, {dt:.1f} s; "
                      "timing-faithful draws (shared atomic sampler cursors)",
            "rays_counted": "built (every Ray constructed, Ray.cpp:25-28)"}


def strip_comments(src):
    """C++ source without its comments and with whitespace runs collapsed: the code a compiler
    sees (string and character literals kept verbatim), so documentation edits leave the kernel
    source stamp unchanged."""
    out, i, n = [], 0, len(src)
    while i < n:
        c = src[i]
        if c in "\"'":
            j = i + 1
            while j < n and src[j] != c:
                j += 2 if src[j] == "\\" else 1
            out.append(src[i:j + 1])
            i = j + 1
        elif src.startswith("//", i):
            j = src.find("\n", i)
            i = n if j < 0 else j
        elif src.startswith("/*", i):
            j = src.find("*/", i + 2)
            i = n if j < 0 else j + 2
            out.append(" ")
        else:
            out.append(c)
            i += 1
    return " ".join("".join(out).split())


def kernel_source_stamp():
    """sha256 of the sources the walk / shading kernels and the walk tree they read are built from
    (the HIP kernels and the host scene build), comments stripped: a PMC profile is reported only
    while it was measured on this exact code."""
    import hashlib
    h = hashlib.sha256()
    d = os.path.join(HERE, "mobileraytracer_amd", "csrc")
    for name in sorted(os.listdir(d)):
        if name.endswith((".hip", ".hpp", ".cpp")):
            with open(os.path.join(d, name), encoding="utf-8") as f:
                h.update(name.encode() + b"\0" + strip_comments(f.read()).encode())
    return h.hexdigest()


PMC_PROFILE = os.path.join("profiles", "r06_pmc_traffic.json")


def workload_key(args, shard_of):
    """What a PMC profile must have measured to be reported on this bench line."""
    return {"width": args.width, "height": args.height, "spp": args.spp, "max_depth": args.max_depth,
            "shader": args.shader, "shard_of": shard_of, "scene": getattr(args, "scene", "conference")}


def pmc_traffic(workload):
    """Bytes beyond L2 per launch for each kernel from the committed rocprofv3 PMC summary
    (tools/pmc_run.sh: FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md),
    used only when its kernel-source stamp equals this build's AND it profiled this workload (else
    traffic null: a profile of other kernels or of another frame size is never reported)."""
    path = os.path.join(HERE, PMC_PROFILE)
    if not os.path.exists(path):
        return {}, {"file": PMC_PROFILE, "status": "absent"}
    with open(path) as f:
        j = json.load(f)
    stamp = kernel_source_stamp()
    if j.get("kernel_source_sha256") != stamp:
        return {}, {"file": PMC_PROFILE, "status": "stale (measured on other kernel sources)",
                    "profile_sha256": j.get("kernel_source_sha256"), "build_sha256": stamp}
    if j.get("workload") != workload:
        return {}, {"file": PMC_PROFILE, "status": "other workload (profiled: %s)" % (j.get("workload"),)}
    return j.get("bytes_beyond_l2_per_launch", {}), {"file": PMC_PROFILE, "status": "current",
                                                     "kernel_source_sha256": stamp, "workload": workload,
                                                     "counters": j.get("counters", {})}


# MI355X: 256 CUs in 8 XCDs, 4 SIMDs per CU; a wave64 VALU instruction holds its SIMD 4 cycles
N_CUS, N_XCDS, SIMDS_PER_CU = 256, 8, 4


def issue_fractions(ctr):
    """Instruction issue of one kernel from its PMC averages (per launch): VALU = wave64 VALU
    instructions x 4 cycles over the SIMD-cycles of the launch (GRBM_GUI_ACTIVE is summed over the 8
    XCDs), SALU = scalar instructions over the CU-cycles (one scalar unit per CU), lane use = active
    lanes per issued VALU instruction.  None where a counter is missing."""
    cyc = ctr.get("GRBM_GUI_ACTIVE")
    if not cyc:
        return None
    per_xcd = cyc / N_XCDS
    out = {}
    if "SQ_INSTS_VALU" in ctr:
        out["valu_issue"] = ctr["SQ_INSTS_VALU"] * 4.0 / (N_CUS * SIMDS_PER_CU * per_xcd)
    if "SQ_INSTS_SALU" in ctr:
        out["salu_issue"] = ctr["SQ_INSTS_SALU"] / (N_CUS * per_xcd)
    if "SQ_THREAD_CYCLES_VALU" in ctr and ctr.get("SQ_ACTIVE_INST_VALU"):
        out["valu_lane_use"] = ctr["SQ_THREAD_CYCLES_VALU"] / (64.0 * ctr["SQ_ACTIVE_INST_VALU"])
    if "TD_TD_BUSY" in ctr:
        out["td_busy"] = ctr["TD_TD_BUSY"] / (N_CUS * per_xcd)
    return out or None


def kernel_roofline(r, step, overlap=1):
    """Per-kernel algorithmic bytes and serialised launch durations (outside the timed region).

    Kernels as the timed frames run them: level 1's camera rays are packet-walked by k_trace_packet
    (or, with tuning key 17, generated, walked and shaded in one launch, k_trace_packet_shade);
    k_trace is the per-lane closest-hit walk of levels 2 .. maxDepth (level maxDepth + 1 is not
    walked); k_shade shades levels 1 (2 when fused) .. maxDepth; k_shadow walks the shadow rays of
    every level.  Bytes per level come from one counting frame (which runs level
    1 as separate launches: the same walk, counted), durations from two frames with the shadow
    stream serialised and HIP events around every launch on the stream it runs on."""
    r.set_profiling(counting=True)
    step()
    c = r.frame_stats()
    keys = ("traceMs", "shadowMs", "shadeMs", "fusedMs", "traceLaunches", "shadowLaunches", "shadeLaunches",
            "fusedLaunches")
    frames = 2

    def timed_frames(overlap):
        r.set_tuning(3, overlap)  # 0: shadow rays on the render stream, every launch timed alone
        r.set_profiling(timing=True)
        t = dict.fromkeys(keys, 0)
        t["level1TraceMs"] = 0.0  # level 1's walk: the packet kernel where it is not fused with its shading
        for _ in range(frames):
            step()
            f = r.frame_stats()
            for k in keys:
                t[k] += f[k]
            t["level1TraceMs"] += f["levelTraceMs"][0]
        r.set_profiling()
        return t

    t = timed_frames(0)
    # the same launches in product frames (the shadow walk beside the next level's walk and shading):
    # each launch's time on its own stream, stretched by what shares the GPU with it.  (With
    # --overlap 0 the product frames are the serialised ones: no second pass, so a rocprofv3 summary of
    # such a run holds only serialised launches and recomputes avg_launch_ms.)
    t_ov = timed_frames(1) if overlap else t
    r.set_tuning(3, 1)
    md = r.config.maxDepth
    rays = c["levelRays"]          # index l - 1: rays of depth l
    shadows = c["levelShadowRays"]
    nodes, tris, leaves = c["levelNodeRecords"], c["levelTriTests"], c["levelLeafRecords"]
    shaded = c["levelShadedVertices"]
    fused = t["fusedLaunches"] > 0
    packet = not fused and r.get_tuning(16) != 0  # level 1 by the packet walk in its own launch
    # k_trace: depths 2 .. maxDepth (depth 1: the packet walk, fused or not), 1 .. without packets
    walk_levels = range(1 if (fused or packet) else 0, md)
    # k_trace: per ray 32 (ray read: origin, direction) + 16 (hit write) + 32 per node record + 36 per
    # triangle test; `fetched`: the bytes the load instructions request - 16 per child
    # record of the quantized 4-wide tree, 48 per walk-tree leaf record (exact box + certified-cull
    # record), 36 per triangle test (three 12-B loads: A, AB, AC)
    trace_b = sum(48.0 * rays[l] + 32.0 * nodes[l] + 36.0 * tris[l] for l in walk_levels)
    trace_f = sum(48.0 * rays[l] + 16.0 * nodes[l] + 48.0 * leaves[l] + 36.0 * tris[l] for l in walk_levels)
    # k_shadow: 32 (ray read) + 4 (flag write) + the same gathers
    n_sh = c["shadowRays"]
    shadow_b = 36.0 * n_sh + 32.0 * c["shadowNodeRecords"] + 36.0 * c["shadowTriTests"]
    shadow_f = 36.0 * n_sh + 16.0 * c["shadowNodeRecords"] + 48.0 * c["shadowLeafRecords"] + 36.0 * c["shadowTriTests"]

    # shading of depth l: per ray 52 read (origin, direction, hit, tree code) + 16
    # written (vertex or result record); per shaded hit 48 (normals, material id) + 64 (material) + 64
    # (light) + 32 (the vertex's six draws, one compact block); per shadow ray 48 written; per child ray
    # 36 written (not for the depth-capped level's children, whose payloads are never written)
    # (read_rays False: the fused level-1 kernel, whose rays and hits stay in registers; regen: level 1's
    # k_shade regenerating its camera rays (tuning key 33 = 2): it reads the hit only, 16 + 16 per ray)
    def shade_bytes(l, read_rays=True, regen=False):
        child = 36.0 * rays[l + 1] if l + 1 < md else 0.0
        per_ray = 32.0 if regen else 68.0 if read_rays else 16.0
        return per_ray * rays[l] + 208.0 * shaded[l] + 48.0 * shadows[l] + child

    shade_levels = range(1 if fused else 0, md)
    gen = r.get_tuning(33) if packet else 0  # 1: the packet walk generates and stores the camera rays; 2: k_shade regenerates them
    shade_b = sum(shade_bytes(l, regen=(l == 0 and gen == 2)) for l in shade_levels)
    # the fused level-1 launch: the packet walk's gathers (no ray record read: the rays are generated
    # in the kernel; no hit record written: it is shaded in the same wave) + level 1's shading
    fused_b = 32.0 * nodes[0] + 36.0 * tris[0] + shade_bytes(0, read_rays=False)
    fused_f = 16.0 * nodes[0] + 48.0 * leaves[0] + 36.0 * tris[0] + shade_bytes(0, read_rays=False)

    def entry(frame_bytes, ms, launches, fetched_bytes=None, levels=None, ms_ov=None):
        launches_pf = launches / frames
        per_launch = frame_bytes / max(1.0, launches_pf)
        avg_ms = ms / max(1, launches)
        ach = per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        e = {"algorithmic_bytes_per_launch": per_launch, "avg_launch_ms": avg_ms, "launches_per_frame": launches_pf,
             "achieved": ach, "peak": PEAK_VMEM_GBS, "unit": "GB/s", "frac": ach / PEAK_VMEM_GBS}
        if ms_ov is not None and ms_ov > 0:
            # the product frames' launches (overlapped streams; what rocprofv3 sees in the timed frames)
            avg_ov = ms_ov / max(1, launches)
            e.update({"avg_launch_ms_overlapped": avg_ov,
                      "frac_overlapped": per_launch / (avg_ov * 1e-3) / 1e9 / PEAK_VMEM_GBS})
        if levels is not None:
            e["depths"] = levels
        if fetched_bytes is not None:
            f = fetched_bytes / max(1.0, launches_pf)
            fa = f / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
            e.update({"fetched_bytes_per_launch": f, "achieved_fetched": fa, "frac_fetched": fa / PEAK_VMEM_GBS})
        return e

    walked = sum(rays[l] for l in walk_levels)
    per_ray = {"nodes": sum(nodes[l] for l in walk_levels) / max(1, walked),
               "tris": sum(tris[l] for l in walk_levels) / max(1, walked),
               "leaves": sum(leaves[l] for l in walk_levels) / max(1, walked),
               "camera_nodes": nodes[0] / max(1, rays[0]), "camera_tris": tris[0] / max(1, rays[0]),
               "shadow_nodes": c["shadowNodeRecords"] / max(1, n_sh),
               "shadow_tris": c["shadowTriTests"] / max(1, n_sh),
               "shadow_leaves": c["shadowLeafRecords"] / max(1, n_sh), "shaded_vertices": c["shadedVertices"]}
    lv = lambda rng: [l + 1 for l in rng]  # noqa: E731
    # level 1 unfused: its packet walk (k_trace_packet) reads the camera rays k_raygen wrote and writes
    # the hits; its time is the first level's trace time, its launches one per frame
    packet_ms = t["level1TraceMs"] if packet else 0.0
    packet_ms_ov = t_ov["level1TraceMs"] if packet else 0.0
    packet_launches = frames if packet else 0
    out = {"k_trace": entry(trace_b, t["traceMs"] - packet_ms, t["traceLaunches"] - packet_launches, trace_f,
                            lv(walk_levels), t_ov["traceMs"] - packet_ms_ov),
           "k_shadow": entry(shadow_b, t["shadowMs"], t["shadowLaunches"], shadow_f, None, t_ov["shadowMs"]),
           "k_shade": entry(shade_b, t["shadeMs"], t["shadeLaunches"] - t["fusedLaunches"], None, lv(shade_levels),
                            t_ov["shadeMs"])}
    if fused:
        out["k_trace_packet_shade"] = entry(fused_b, t["fusedMs"], t["fusedLaunches"], fused_f, [1])
        out["k_trace_packet_shade"]["frac_basis"] = ("per lane (SURVEY 8(d)); the packet fetches nodes, leaf and "
                                                     "triangle records once per wave: not a memory roofline")
    elif packet:
        # The packet walk fetches each node (128 B: the float grid-index copy), leaf record (48 B) and
        # triangle record (48 B) ONCE per wave through the scalar cache (mrt_trace_packet.hpp), not per
        # lane: priced by what it moves - per lane the ray read (32 B), the hit write (16 B) and the
        # winner's triangle re-read for u, v (48 B); per wave the records it loads (counting frame,
        # packetWaveRecords).  SURVEY 8(d)'s per-lane price is kept beside it as `lane_basis_*`.
        # (tuning key 33: 1 the walk generates the rays and stores their 36-B records instead of reading
        # 32 B; 2 it stores nothing, k_shade regenerates them)
        wn, wl, wt = c["packetWaveRecords"]
        ray_b = 32.0 if gen == 0 else 36.0 if gen == 1 else 0.0
        packet_b = (64.0 + ray_b) * rays[0] + 128.0 * wn + 48.0 * wl + 48.0 * wt
        lane_b = 48.0 * rays[0] + 32.0 * nodes[0] + 36.0 * tris[0]
        e = entry(packet_b, packet_ms, packet_launches, None, [1], packet_ms_ov)
        e["frac_basis"] = ("bytes the kernel moves: per lane 64 B (hit, winner's triangle) + the camera ray's record "
                           f"({ray_b:.0f} B: tuning key 33 = {gen}), per wave 128 B per node visit + 48 B per leaf "
                           "record + 48 B per triangle record (scalar loads, once per wave)")
        lpf = max(1.0, packet_launches / frames)  # packet launches per frame (the counting frame is one frame)
        e["wave_records_per_launch"] = {"node_visits": wn / lpf, "leaf_records": wl / lpf, "triangle_records": wt / lpf}
        e["lane_basis_bytes_per_launch"] = lane_b / lpf
        e["lane_basis_frac"] = (e["lane_basis_bytes_per_launch"] / (e["avg_launch_ms"] * 1e-3) / 1e9 / PEAK_VMEM_GBS
                                if e["avg_launch_ms"] > 0 else 0.0)
        e["lane_basis_note"] = ("SURVEY 8(d)'s per-lane price of every node / triangle a lane passes; the packet never "
                                "moves these bytes per lane, so this is not a memory-roofline fraction")
        out["k_trace_packet"] = e
    return out, per_ray


def main():
    args = parse()
    import torch
    action, what = launch_plan(args.gpus, os.environ, torch.cuda.device_count(), args.path)
    if action == "error":
        print(f"bench.py: {what}", file=sys.stderr, flush=True)
        sys.exit(2)
    if action == "spawn":
        sys.exit(spawn_ranks(what, sys.argv[1:]))
    import torch.distributed as dist
    import mobileraytracer_amd as m
    from mobileraytracer_amd import scenes

    group = group_devices(args.gpus, os.environ) if args.path == "group" else []
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MRT_BENCH_BACKEND=gloo (rehearsal only: several ranks sharing one GPU, gather through host
    # memory); the measured multi-GPU path is RCCL ("nccl") with one GPU per rank
    backend = os.environ.get("MRT_BENCH_BACKEND", "nccl")
    # MRT_BENCH_FORCE_DIST=1 (rehearsal only): the multi-GPU path (process group, packed shard,
    # gather, unpack) even at world size 1, so a one-GPU box exercises the RCCL calls
    dist_on = world > 1 or os.environ.get("MRT_BENCH_FORCE_DIST") == "1"
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        local = local % torch.cuda.device_count() if backend == "gloo" else local
        torch.cuda.set_device(local)
    else:
        torch.cuda.set_device(group[0] if group else 0)
    scene = scenes.conference() if args.scene == "conference" else scenes.conference_flat()
    shard_of = args.shard_of if (args.shard_of > 1 and not dist_on and len(group) <= 1) else 0
    cfg = m.Config(width=args.width, height=args.height, shader=args.shader, sceneIndex=-1,
                   samplesPixel=args.spp, samplesLight=1, maxDepth=args.max_depth, objFilePath=scene[0],
                   mtlFilePath=scene[1], camFilePath=scene[2], rankIndex=rank,
                   rankCount=shard_of if shard_of else world, device=torch.cuda.current_device(),
                   devices=group if len(group) > 1 else [])
    # (the renderer checks at creation that its render and shadow streams run concurrently, whatever
    # streams RCCL or torch created: DESIGN.md section 6)
    r = m.Renderer(cfg)
    if dist_on:
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    r.set_tuning(3, args.overlap)
    # MRT_BENCH_TUNING="17=0,...": tuning keys for profiling runs (tools/pmc_run.sh profiles the
    # timed frames with level 1 unfused, so that its PMC averages cover the same walk launches as
    # the serialised roofline frames)
    for kv in filter(None, os.environ.get("MRT_BENCH_TUNING", "").split(",")):
        k, v = kv.split("=")
        r.set_tuning(int(k), int(v))
    info = r.scene_info()
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    slots_max = info["pixelSlotsMax"]
    bitmap = torch.zeros(args.width * args.height, dtype=torch.int32, device="cuda")
    packed = torch.zeros(slots_max, dtype=torch.int32, device="cuda")
    gathered = torch.zeros((world, slots_max), dtype=torch.int32, device="cuda") if rank == 0 else None

    # Single-process frames run on the renderer's own stream (stream 0), as RayTrace renders: a
    # caller's stream costs a join event per frame (the frame then waits for the caller's earlier
    # work); the buffers are settled by torch.cuda.synchronize() before and after every timed loop.
    # The RCCL path keeps torch's stream (the gather follows the frame on it), and so does the loop
    # that copies every frame to the host (each frame after the previous frame's copy).
    def step(own=0):
        if shard_of:
            r.render_frame_device(0, packed.data_ptr(), own)
        elif not dist_on:
            r.render_frame_device(bitmap.data_ptr(), 0, own)
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

    torch.cuda.synchronize()  # (the buffers' fills on torch's stream, before frames on the renderer's)
    for _ in range(args.warmup):
        step()
    kernels, per_ray = kernel_roofline(r, step, args.overlap)
    r.set_tuning(3, args.overlap)

    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    rays0 = r.get_total_casted_rays()
    walked = 0  # closest-hit rays traversed + shadow rays: the rays whose walk ran
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        w, sr = r.frame_rays()  # (frame_stats()'s dict costs ~20 us of Python per frame)
        walked += w + sr
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    rays = r.get_total_casted_rays() - rays0

    # BASELINE.md section 2's timed window ends with the bitmap in host memory: a second, shorter
    # timed loop adds the D2H copy of the frame into pinned host memory to every frame
    host_bm = torch.empty(bitmap.numel(), dtype=torch.int32, pin_memory=True) if rank == 0 else None
    if dist_on:
        dist.barrier()
    k2 = max(1, min(args.steps, 10))
    t2 = time.perf_counter()
    for _ in range(k2):
        step(sh)  # (on torch's stream: each frame after the previous frame's copy)
        if rank == 0:
            host_bm.copy_(bitmap, non_blocking=True)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    d2h_ms = (time.perf_counter() - t2) / k2 * 1e3

    # median of 5 frames, each timed alone (synchronised on both sides)
    singles = []
    for _ in range(5):
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        singles.append((time.perf_counter() - t3) * 1e3)
    median5_ms = sorted(singles)[2]

    if dist_on:
        red = "cpu" if backend == "gloo" else "cuda"
        t = torch.tensor([elapsed], dtype=torch.float64, device=red)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        t = torch.tensor([median5_ms], dtype=torch.float64, device=red)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        median5_ms = float(t.item())
        n = torch.tensor([rays, walked], dtype=torch.float64, device=red)
        dist.all_reduce(n, op=dist.ReduceOp.SUM)
        rays, walked = [int(x) for x in n.tolist()]

    if rank != 0:
        dist.destroy_process_group()
        return

    frames = max(1, args.steps)
    n_gpus = len(group) if group else world
    traffic, traffic_src = pmc_traffic(workload_key(args, shard_of)) if n_gpus == 1 else (
        {}, {"status": "not collected for N > 1"})
    counters = traffic_src.pop("counters", {})
    for name, e in kernels.items():
        tb = traffic.get(name)
        e["traffic"] = tb
        e["hbm_frac"] = (tb / (e["avg_launch_ms"] * 1e-3) / 1e9 / PEAK_HBM_GBS) if tb and e["avg_launch_ms"] > 0 else None
        # what bounds a walk that is not byte-bound: instruction issue (PMC, same profile as `traffic`)
        e["issue"] = issue_fractions(counters[name]) if name in counters else None
    dom = kernels["k_trace"]
    out = {
        "metric": BASELINE_METRIC,
        "value": walked / elapsed / 1e6,
        "unit": "Mrays/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / frames * 1e3,
        # the same frames with the bitmap copied to pinned host memory after each (the reference's
        # timed window includes it); `value` excludes it
        "ms_per_step_with_d2h": d2h_ms,
        "value_with_d2h": (walked / frames) / (d2h_ms * 1e-3) / 1e6 if d2h_ms else None,
        # BASELINE.md section 2's statistic: the median of 5 single frames (max over ranks)
        "ms_per_step_median5": median5_ms,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic" if scenes.is_standin(scene[0]) else "conference.obj",
        "config": {
            "workload": ("conference" if args.scene == "conference" else "conference_flat") +
                        f"_{args.width}x{args.height}_{args.spp}spp_pathtracer_depth{args.max_depth}",
            "scene": (("conference stand-in" if args.scene == "conference" else
                       "flat-geometry conference stand-in (large flat triangles, slivers, coplanar panels)") +
                      ": 331179 triangles + 2 area lights, reference conference.mtl/.cam "
                      "(conference.obj is absent from the reference snapshot)") if scenes.is_standin(scene[0])
            else scene[0],
            "resolution": [args.width, args.height],
            "rendered_pixels": int(info["pixelSlots"]) if world == 1 else None,
            "devices": group if group else None,
            "spp": args.spp, "max_depth": args.max_depth, "samples_light": 1,
            "shader": "PathTracer" if args.shader == 2 else "Whitted",
            "parallelism": (f"screen-tile shard x{world} + " + ("RCCL gather" if backend == "nccl" else "gloo gather (rehearsal)"))
            if dist_on else (f"device group x{len(group)}: one process, one shard worker per GPU, peer-copy assembly"
                             + (" (repeated ordinals: rehearsal on one GPU)" if len(set(group)) < len(group) else ""))
            if len(group) > 1 else (f"rank 0's shard of a {shard_of}-GPU frame, on one GPU (rehearsal)" if shard_of
                             else "single GPU"),
            "rays_walked_per_frame": walked / frames,
            "rays_built_per_frame": rays / frames,
            "mrays_per_s_built": rays / elapsed / 1e6,
            "value_counts": "walked rays (closest-hit walks run + shadow rays)",
            "event_timing_in_timed_frames": False,
        },
        "roofline": {
            # the walk is bound by the per-CU vector-memory path serving divergent gathers of a
            # cache-resident scene (PMC: texture-data unit busy ~92 %, bytes beyond L2 ~11 % of the
            # algorithmic bytes; profiles/), not by HBM
            "bound": "vmem-gather",
            "kernel": "k_trace (closest hit, per-lane walk of depths %s)" % dom.get("depths"),
            "achieved": dom["achieved"],
            "peak": PEAK_VMEM_GBS,
            "unit": "GB/s",
            "frac": dom["frac"],
            "traffic": dom["traffic"],
            "traffic_source": traffic_src,
            # the same launch priced at the bytes its loads request (16 B per quantized child record,
            # 48 B per leaf record, 36 B per triangle test) instead of SURVEY 8(d)'s 32 B per record
            "frac_fetched": dom["frac_fetched"],
            "achieved_fetched": dom["achieved_fetched"],
            "avg_launch_ms": dom["avg_launch_ms"],
            "algorithmic_bytes_per_launch": dom["algorithmic_bytes_per_launch"],
            "per_ray": per_ray,
            "peak_source": "MI355X_MICROARCH.md: L2 34.5 TB/s aggregate, 36.9 TB/s with L1 reuse",
            # measured on MI355X by tools/gather_ceiling.hip (profiles/r02_gather_ceiling.jsonl): dependent
            # 64-byte record chains from a 32 MiB table, every lane at a different record vs every lane of
            # a wave at the same one; the walk's rays sit between the two (coherent camera rays, scattered
            # bounces)
            "measured_ceilings_gbs": {"divergent_64B_records_32MiB": 6648.4, "wave_coherent_64B_records_32MiB": 27859.6},
            "durations": "serialised frames (shadow stream off), HIP events on the render stream",
            # the same kernel in the product frames (shadow walks beside it): slower per launch
            "frac_overlapped": dom.get("frac_overlapped"),
            "avg_launch_ms_overlapped": dom.get("avg_launch_ms_overlapped"),
            # the rocprofv3 summaries these durations agree with (tools/final.sh): a run whose frames are
            # all serialised (--overlap 0) for avg_launch_ms, the default run for the overlapped figure
            "rocprof_summaries": {"serialised": "profiles/r06_kernel_stats_serial.csv",
                                  "product_frames": "profiles/r06_kernel_stats.csv"},
            "kernels": kernels,
        },
        "cpu_baseline": None,
        # the loaded library was built from the sources in this tree (Makefile stamp)
        "library_build_current": m._native.build_is_current(),
    }
    if n_gpus == 1 and not shard_of and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, scene)
    print(json.dumps(out), flush=True)
    if args.dump_bitmap:
        import numpy as np
        np.save(args.dump_bitmap, bitmap.cpu().numpy())
    r.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
