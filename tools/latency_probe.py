"""Latency of the walks for a handful of rays on an otherwise idle GPU: shadow rays from random
floor points to the light panel and closest-hit rays from the floor into the upper hemisphere (the
scene's own kinds of rays), in batches of 64 .. 64k, per tuning setting (wall clock around
mrt_trace_rays, which is synchronous: median of 7).

    python tools/latency_probe.py ["8=0" "16=0+8=0" ...]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mobileraytracer_amd as m  # noqa: E402
from mobileraytracer_amd import scenes  # noqa: E402


def rays(n, rng):
    p = np.stack([rng.uniform(-1100, 1100, n), np.full(n, 1.0), rng.uniform(-1300, 1300, n)], 1).astype(np.float32)
    tgt = np.stack([rng.uniform(-300, 300, n), np.full(n, 1030.0), rng.uniform(-420, 420, n)], 1).astype(np.float32)
    sd = tgt - p
    dist = np.linalg.norm(sd, axis=1).astype(np.float32)
    sd = (sd / dist[:, None]).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d[:, 1] = np.abs(d[:, 1])
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    return p, sd, dist, d


def main():
    o, l, c = scenes.conference()
    cfg = m.Config(width=64, height=64, shader=1, sceneIndex=-1, objFilePath=o, mtlFilePath=l, camFilePath=c)
    r = m.Renderer(cfg)
    settings = sys.argv[1:] or ["default"]
    for st in settings:
        for kv in filter(None, st.split("+")):
            if kv != "default":
                k, v = kv.split("=")
                r.set_tuning(int(k), int(v))
        sizes = [int(x) for x in os.environ.get("SIZES", "64,640,6400,64000").split(",")]
        for n in sizes:
            p, sd, dist, d = rays(n, np.random.default_rng(n))
            if os.environ.get("MISS") == "1":  # rays that miss the scene box: the launch alone
                p = p + np.float32(1e5)
                d = np.abs(d)
            ts, tc = [], []
            for _ in range(7):
                t0 = time.perf_counter()
                r.trace_rays(p, sd, dist=dist, any_hit=True)
                t1 = time.perf_counter()
                r.trace_rays(p, d)
                t2 = time.perf_counter()
                ts.append(t1 - t0)
                tc.append(t2 - t1)
            print(f"{st:>12} n={n:6d} shadow {np.median(ts) * 1e6:8.1f} us  closest {np.median(tc) * 1e6:8.1f} us", flush=True)
        for kv in filter(None, st.split("+")):  # back to the defaults
            if kv != "default":
                k, _ = kv.split("=")
                r.set_tuning(int(k), {"8": 1, "16": 1, "9": 0, "5": 1}.get(k, 0))
    r.close()


main()
