"""First GPU run: render the configs, save outputs under gpurun_out/first_light for offline parity."""
import os, sys, time, json
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mobileraytracer_amd as m
from mobileraytracer_amd import scenes
out = os.path.join("gpurun_out", "first_light"); os.makedirs(out, exist_ok=True)
res = {}
def run(name, cfg, frames=1, prof=False):
    t0 = time.time(); r = m.Renderer(cfg); tc = time.time() - t0
    info = r.scene_info()
    bm = np.zeros(cfg.width * cfg.height, np.int32)
    r.render_frame(bm)  # warmup
    if prof: r.set_profiling(timing=True)
    t0 = time.time()
    for _ in range(frames): r.render_frame(bm)
    dt = (time.time() - t0) / frames
    st = r.frame_stats()
    np.save(os.path.join(out, name + ".npy"), bm)
    rays = st["rays"] + st["shadowRays"]
    res[name] = dict(create_s=tc, frame_ms=dt * 1e3, rays=rays, mrays=rays / dt / 1e6, info=info, stats=st)
    print(name, json.dumps(res[name]), flush=True)
    k, i, t = r.primary_hits(); np.savez(os.path.join(out, name + "_hits.npz"), kind=k, index=i, t=t)
    r.close()
run("cornell_whitted_256", m.Config(width=256, height=256, shader=1, sceneIndex=0))
run("cornell_whitted_512", m.Config(width=512, height=512, shader=1, sceneIndex=0))
run("cornell_pt_256_4spp", m.Config(width=256, height=256, shader=2, sceneIndex=0, samplesPixel=4))
o, l, c = scenes.cornell_water()
run("water_pt_128_4spp", m.Config(width=128, height=128, shader=2, sceneIndex=-1, samplesPixel=4, objFilePath=o, mtlFilePath=l, camFilePath=c))
run("water_whitted_128", m.Config(width=128, height=128, shader=1, sceneIndex=-1, objFilePath=o, mtlFilePath=l, camFilePath=c))
o, l, c = scenes.conference()
run("conf_whitted_1080", m.Config(width=1920, height=1080, shader=1, sceneIndex=-1, objFilePath=o, mtlFilePath=l, camFilePath=c), frames=3, prof=True)
run("conf_pt_1080_4spp", m.Config(width=1920, height=1080, shader=2, sceneIndex=-1, samplesPixel=4, maxDepth=5, objFilePath=o, mtlFilePath=l, camFilePath=c), frames=3, prof=True)
json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
