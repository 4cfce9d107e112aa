"""Does splitting a shard into two concurrently rendered halves fill the level tails?

For N in NS (default 1, 8): rank 0's shard of an N-way C4 frame rendered by one renderer, against
the same amount of work as two renderers - ranks 0 and N of a 2N-way partition - each rendering its
half from a host thread of its own on the same GPU (own streams, own queues), so that one half's
level tails overlap the other's bulk.  Frame times are per frame of the pair (both halves done).
    python tools/pipeline_probe.py            (env NS="1 8", FRAMES=10, ROUNDS=3)"""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mobileraytracer_amd as m  # noqa: E402
from mobileraytracer_amd import scenes  # noqa: E402


def make(rank, count):
    o, l, c = scenes.conference() if os.environ.get("SCENE", "conference") == "conference" else scenes.conference_flat()
    cfg = m.Config(width=1920, height=1080, shader=2, sceneIndex=-1, samplesPixel=4, maxDepth=5, objFilePath=o,
                   mtlFilePath=l, camFilePath=c, rankIndex=rank, rankCount=count)
    r = m.Renderer(cfg)
    buf = torch.zeros(max(1, r.scene_info()["pixelSlotsMax"]), dtype=torch.int32, device="cuda")
    return r, buf


def frames(r, buf, k):
    for _ in range(k):
        r.render_frame_device(0, buf.data_ptr(), 0)


def main():
    k = int(os.environ.get("FRAMES", 10))
    for n in [int(x) for x in os.environ.get("NS", "1 8").split()]:
        single = make(0, n)
        pair = [make(0, 2 * n), make(n, 2 * n)]
        frames(*single, 2)
        for p in pair:
            frames(*p, 2)
        torch.cuda.synchronize()
        res = {"single": [], "pair": []}
        for _ in range(int(os.environ.get("ROUNDS", 3))):
            t0 = time.perf_counter()
            frames(*single, k)
            torch.cuda.synchronize()
            res["single"].append((time.perf_counter() - t0) / k * 1e3)
            th = [threading.Thread(target=frames, args=(p[0], p[1], k)) for p in pair]
            t0 = time.perf_counter()
            for t in th:
                t.start()
            for t in th:
                t.join()
            torch.cuda.synchronize()
            res["pair"].append((time.perf_counter() - t0) / k * 1e3)
        print(f"N={n}: single shard {min(res['single']):.3f} ms (rounds {[round(x, 3) for x in res['single']]}), "
              f"two concurrent halves {min(res['pair']):.3f} ms (rounds {[round(x, 3) for x in res['pair']]})",
              flush=True)
        for r, _ in [single] + pair:
            r.close()


if __name__ == "__main__":
    main()
